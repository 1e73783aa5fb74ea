"""FP8 W8A8 quantization on the CPU (ops/quant.py reference path; SURVEY §2.8 quantization row).

The reference only documents quantization (bitsandbytes int8/int4 + absmax fallback,
``plan.md:109-112,438-456``); there is no reference output to pin against, so parity is
unpinned and these tests check the scheme's own invariants."""
import pytest
import torch

from distributed_llms_amd import ops
from distributed_llms_amd.config import EngineConfig
from distributed_llms_amd.engine.llm_engine import LLMEngine, build_stage
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.ops import quant


def test_weight_quantization_is_per_channel_absmax():
    w = torch.randn(64, 96)
    w[3] *= 100                                   # one loud channel does not crush the others
    fw = quant.quantize_weight(w)
    assert fw.q.dtype == torch.float8_e4m3fn and fw.scale.shape == (64,)
    torch.testing.assert_close(fw.scale, w.abs().amax(1) / 448.0)
    assert fw.q.float().abs().amax(1).eq(448.0).all()        # every row uses the full range
    rel = (fw.dequantize() - w).norm(dim=1) / w.norm(dim=1)
    assert rel.max() < 0.04
    assert fw.nbytes() == 64 * 96 + 64 * 4


def test_zero_rows_quantize_to_zero_with_unit_scale():
    x = torch.zeros(3, 16)
    x[1] = torch.linspace(-2, 2, 16)
    q, s = quant.quantize_rows_ref(x)
    assert s[0] == 1 and s[2] == 1 and q[0].float().abs().sum() == 0
    assert q[1].float().abs().max() == 448.0


@pytest.mark.parametrize("swiglu", [False, True])
def test_linear_dispatches_fp8_weights(swiglu):
    torch.manual_seed(0)
    x, w = torch.randn(5, 64), torch.randn(32, 64) * 0.1
    fw = quant.quantize_weight(w)
    y = ops.linear_swiglu(x, fw) if swiglu else ops.linear(x, fw)
    ref = x @ w.t()
    if swiglu:
        g, u = ref.chunk(2, -1)
        ref = torch.nn.functional.silu(g) * u
    assert ((y - ref).norm() / ref.norm()) < 0.08
    with pytest.raises(ValueError):
        ops.linear(x, fw, bias=torch.zeros(32))


def test_stage_quantize_converts_projections_and_experts():
    ecfg = EngineConfig(model="tiny-mixtral", dtype="float32", device="cpu", quant="fp8")
    s = build_stage(ecfg)
    lw = s.layers[0]
    assert isinstance(lw["wqkv"], quant.Fp8Weight) and isinstance(lw["wo"], quant.Fp8Weight)
    assert isinstance(lw["experts_gate_up"], quant.Fp8Experts) and isinstance(lw["experts_down"], quant.Fp8Experts)
    skip = set(quant.QUANT_KEYS) | set(quant.EXPERT_KEYS)
    assert all(isinstance(t, torch.Tensor) for k, t in lw.items() if k not in skip)     # router, norms
    with pytest.raises(ValueError):
        EngineConfig(model="tiny-llama", quant="int3").validate()


def test_fp8_moe_tracks_the_bf16_moe():
    from distributed_llms_amd.ops import moe
    torch.manual_seed(1)
    t, h, i, e = 12, 64, 96, 4
    x = torch.randn(t, h)
    wr, gu, dn = torch.randn(e, h), torch.randn(e, 2 * i, h) * 0.1, torch.randn(e, h, i) * 0.1
    ref = moe.forward(x, wr, gu, dn, 2)
    out = moe.forward(x, wr, quant.quantize_experts(gu), quant.quantize_experts(dn), 2)
    assert ((out - ref).norm() / ref.norm()) < 0.08
    with pytest.raises(TypeError):
        moe.forward(x, wr, quant.quantize_experts(gu), dn, 2)


def test_cpu_engine_runs_fp8():
    base = EngineConfig(model="tiny-llama", dtype="float32", device="cpu", max_batch=4, max_seq_len=64,
                        num_kv_blocks=64, use_graphs=False)
    prompts = [[1, 2, 3, 4], [5, 6, 7]]
    sp = SamplingParams(max_new_tokens=6, ignore_eos=True)
    ref = LLMEngine(base).generate(prompts, sp)
    e8 = LLMEngine(base.apply_overrides(quant="fp8"))
    out = e8.generate(prompts, sp)
    assert [len(o) for o in out] == [6, 6]
    assert [o[0] for o in out] == [o[0] for o in ref]       # first greedy tokens agree
    assert e8.stage.weight_bytes() < LLMEngine(base).stage.weight_bytes() / 2
