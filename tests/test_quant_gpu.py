"""FP8 W8A8 kernels on the GPU (csrc/kernels/quant.hip, gemm_wide.hip ``gemm_wide_fp8``) against
the PyTorch fp32 reference of the same quantized operands (ops/quant.py)."""
import pytest
import torch

from distributed_llms_amd import ops
from distributed_llms_amd.ops import gemm, quant

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _x(m, k, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(m, k, generator=g)
    x *= torch.logspace(-2, 1, m).unsqueeze(1)        # rows over three decades of magnitude
    return x.to(DEV, torch.bfloat16)


@pytest.mark.parametrize("m,k", [(1, 4096), (7, 128), (256, 4096), (64, 14336), (33, 520)])
def test_quant_rows_matches_reference_bit_exact(m, k):
    x = _x(m, k)
    x[0, :] = 0                                           # an all-zero row: scale 1, zeros
    q, s = quant.quantize_rows(x)
    qr, sr = quant.quantize_rows_ref(x)
    torch.testing.assert_close(s, sr.to(DEV), rtol=0, atol=0)
    assert torch.equal(q.view(torch.uint8), qr.to(DEV).view(torch.uint8))


def _oracle(x, w, swiglu=False):
    return quant.linear_ref(x.float().cpu().to(torch.bfloat16), quant.Fp8Weight(w.q.cpu(), w.scale.cpu()),
                            swiglu).float()


@pytest.mark.parametrize("m,n,k,swiglu,splits", [
    (1, 256, 512, False, 1),
    (64, 6144, 4096, False, 0),          # qkv_8b, engine split
    (200, 4096, 4096, False, 8),         # o_8b, split-K reduce
    (256, 2048, 4096, True, 1),          # gate|up slice, SwiGLU epilogue
    (256, 2048, 4096, True, 4),          # split-K SwiGLU (splitk_reduce_swiglu)
    (256, 4096, 14336, False, 0),        # down_8b
    (1000, 1024, 1024, False, 1),        # prefill-sized M, several row tiles
    (5000, 1024, 512, True, 0),          # grouped row-tile order (M >= knobs.fp8_group_m), SwiGLU
    (4500, 2048, 1024, False, 0),        # grouped, partial last row tile and group
])
def test_gemm_wide_fp8_matches_reference(m, n, k, swiglu, splits):
    torch.manual_seed(m + n)
    w = quant.quantize_weight((torch.randn(n, k) * 0.02).to(DEV))
    x = _x(m, k, seed=n)
    y = quant.linear_fp8(x, w, swiglu=swiglu, splits=splits).float().cpu()
    ref = _oracle(x, w, swiglu)
    assert y.shape == ref.shape
    err = (y - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-3, err


def test_fp8_deferred_split_feeds_the_fused_norm():
    m, n, k = 256, 4096, 4096
    w = quant.quantize_weight((torch.randn(n, k) * 0.02).to(DEV))
    x = _x(m, k, seed=3)
    part = quant.linear_fp8(x, w, defer=True)
    assert isinstance(part, gemm.SplitKPartial)
    res = torch.randn(m, n, device=DEV).to(torch.bfloat16)
    nw = torch.rand(n, device=DEV).to(torch.bfloat16)
    y, r = ops.fused_add_rms_norm(part, res.clone(), nw, 1e-5)
    full = _oracle(x, w).to(DEV)
    ry, rr = ops.fused_add_rms_norm(full.to(torch.bfloat16), res.clone(), nw, 1e-5)
    torch.testing.assert_close(r.float(), rr.float(), rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(y.float(), ry.float(), rtol=3e-2, atol=3e-2)


def test_fp8_error_vs_bf16_weights_is_quantization_sized():
    """The W8A8 product against the unquantized bf16 one: a few percent relative error (e4m3
    has 3 mantissa bits), not a layout error."""
    m, n, k = 256, 4096, 4096
    wb = (torch.randn(n, k) * 0.02).to(DEV, torch.bfloat16)
    x = _x(m, k, seed=5)
    y = quant.linear_fp8(x, quant.quantize_weight(wb)).float()
    ref = x.float() @ wb.float().t()
    rel = ((y - ref).norm() / ref.norm()).item()
    assert rel < 0.06, rel


def test_fp8_engine_generates_and_tracks_bf16():
    from distributed_llms_amd.config import EngineConfig
    from distributed_llms_amd.engine.llm_engine import build_stage
    ecfg = EngineConfig(model="tiny-llama", max_batch=8, max_seq_len=128, num_kv_blocks=64, use_graphs=True)
    from distributed_llms_amd.engine.llm_engine import LLMEngine
    from distributed_llms_amd.engine.sequence import SamplingParams
    prompts = [[1, 5, 9, 12, 40], [3, 3, 7], [100, 200, 300, 17, 8, 9, 10]]
    sp = SamplingParams(max_new_tokens=8, ignore_eos=True)
    out_b = LLMEngine(ecfg).generate(prompts, sp)
    e8 = LLMEngine(ecfg.apply_overrides(quant="fp8"))
    layer = e8.runner.stage.layers[0]
    assert all(isinstance(layer[k], quant.Fp8Weight) for k in quant.QUANT_KEYS)
    out_8 = e8.generate(prompts, sp)
    assert [len(o) for o in out_8] == [8, 8, 8]
    # random-init weights: greedy paths may split late, the first tokens agree
    assert sum(a[0] == b[0] for a, b in zip(out_b, out_8)) >= 2
    s = build_stage(ecfg.apply_overrides(quant="fp8"), device=DEV)
    assert s.weight_bytes() < build_stage(ecfg, device=DEV).weight_bytes()


@pytest.mark.parametrize("hidden", [4096, 256, 8192])
def test_norm_kernels_emit_the_same_fp8_as_quantizing_their_output(hidden):
    """rms_norm / fused_add_rms_norm / splitk_add_rms_norm with quant_out: bit-identical to the
    bf16 output quantized by quant_fp8_rows (the epilogue rounds to bf16 first)."""
    m = 37
    x = _x(m, hidden, seed=hidden)
    w = (torch.rand(hidden) + 0.5).to(DEV, torch.bfloat16)
    a = ops.rms_norm(x, w, 1e-5, quant_out=True)
    q, s = quant.quantize_rows(ops.rms_norm(x, w, 1e-5))
    assert torch.equal(a.q.view(torch.uint8), q.view(torch.uint8)) and torch.equal(a.scale, s)
    res = _x(m, hidden, seed=1)
    r1, r2 = res.clone(), res.clone()
    a, r1 = ops.fused_add_rms_norm(x, r1, w, 1e-5, quant_out=True)
    y, r2 = ops.fused_add_rms_norm(x, r2, w, 1e-5)
    q, s = quant.quantize_rows(y)
    assert torch.equal(r1, r2)
    assert torch.equal(a.q.view(torch.uint8), q.view(torch.uint8)) and torch.equal(a.scale, s)
    if hidden % 128 == 0:                       # split-K partial input (splitk_add_rms_norm)
        wl = (torch.randn(hidden, 1024, device=DEV) * 0.02).to(torch.bfloat16)
        h_in = _x(m, 1024, seed=2)
        r1, r2 = res.clone(), res.clone()
        a, r1 = ops.fused_add_rms_norm(gemm.linear_wide(h_in, wl, splits=4, defer=True), r1, w, 1e-5, quant_out=True)
        y, r2 = ops.fused_add_rms_norm(gemm.linear_wide(h_in, wl, splits=4, defer=True), r2, w, 1e-5)
        q, s = quant.quantize_rows(y)
        assert torch.equal(r1, r2)
        assert torch.equal(a.q.view(torch.uint8), q.view(torch.uint8)) and torch.equal(a.scale, s)


def test_fp8_act_input_skips_requantization():
    m, n, k = 200, 4096, 4096
    w = quant.quantize_weight((torch.randn(n, k) * 0.02).to(DEV))
    x = _x(m, k, seed=9)
    act = quant.Fp8Act(*quant.quantize_rows(x), x.shape, x.dtype)
    assert torch.equal(quant.linear_fp8(act, w), quant.linear_fp8(x, w))
    assert quant.fp8_plan(m, n, k) == (4, 128)                      # the two-row-tile split plan
    assert quant.fp8_plan(256, 6144, 4096) == (2, 128)


@pytest.mark.parametrize("t", [5, 64, 256, 300])
def test_fp8_moe_matches_reference(t):
    """Grouped fp8 expert GEMMs (decode, t <= 256) and the per-expert fp8 prefill path against
    quant.moe_mlp_ref on the same quantized experts."""
    from distributed_llms_amd.ops import moe, reference as R
    torch.manual_seed(t)
    h, i, e, k = 256, 384, 8, 2
    x = (torch.randn(t, h) * 0.5).to(DEV, torch.bfloat16)
    wr = (torch.randn(e, h) * 0.1).to(DEV, torch.bfloat16)
    gu = quant.quantize_experts((torch.randn(e, 2 * i, h) * 0.05).to(DEV))
    dn = quant.quantize_experts((torch.randn(e, h, i) * 0.05).to(DEV))
    out = moe.forward(x, wr, gu, dn, k).float().cpu()
    tw, tid = R.moe_route(R.linear(x.float().cpu(), wr.float().cpu()), k)
    ref = quant.moe_mlp_ref(x.cpu(), quant.Fp8Experts(gu.q.cpu(), gu.scale.cpu()),
                            quant.Fp8Experts(dn.q.cpu(), dn.scale.cpu()), tw, tid).float()
    err = (out - ref).abs().max().item()
    assert err <= 3e-2 * ref.abs().max().item() + 1e-3, err
