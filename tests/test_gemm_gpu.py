"""Decode / prefill GEMM kernels (gemm_wide, gemm_sq, gemm_pp, split-K reducers) vs a plain fp32
PyTorch GEMM of the same operands."""
import os
import pytest
import torch
import torch.nn.functional as F

from distributed_llms_amd import ops
from distributed_llms_amd.ops import gemm

pytestmark = pytest.mark.gpu


def _bf(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


@pytest.mark.parametrize("m", [1, 5, 32, 33, 64])
@pytest.mark.parametrize("n,k", [(6144, 4096), (4096, 4096), (4096, 14336), (128, 768), (2304, 768)])
def test_small_m_linear_dispatch(cuda, m, n, k):
    """Decode batches 1..64 take the wide kernel's 64-row tile through the default dispatch."""
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    assert gemm._use_wide(m, n, k, x, w)
    y = gemm.linear(x, w)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


def test_bias_uses_library_gemm(cuda):
    x, w, b = _bf(9, 768), _bf(2304, 768, scale=0.05), _bf(2304)
    y = gemm.linear(x, w, b)
    ref = x.float() @ w.float().t() + b.float()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [1, 16, 64, 200, 240, 256])
@pytest.mark.parametrize("inter,k", [(14336, 4096), (28672, 8192), (512, 256), (1024, 512)])
def test_small_m_swiglu(cuda, m, inter, k):
    x, w = _bf(m, k), _bf(2 * inter, k, scale=0.05)
    y = gemm.linear_swiglu(x, w)
    gu = x.float() @ w.float().t()
    ref = F.silu(gu[:, :inter]) * gu[:, inter:]
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


def test_large_m_uses_hand_written_prefill_gemm(cuda):
    x, w = _bf(300, 256), _bf(512, 256, scale=0.05)          # a qkv-like (N > K) projection
    assert not gemm._use_wide(300, 512, 256, x, w)
    assert gemm._use_pp(300, 512, 256, x, w, gemm.knobs.K.pp_proj_min_m)
    y = ops.linear(x, w)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


def test_small_m_graph_replay(cuda):
    x, w = _bf(64, 4096), _bf(4096, 4096, scale=0.05)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gemm.linear(x, w)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        y = gemm.linear(x, w)
    for _ in range(3):
        x.copy_(_bf(64, 4096))
        g.replay()
        torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m,n,k", [(256, 4096, 14336), (96, 1024, 8192), (64, 5120, 4096), (32, 8192, 8192)])
def test_deferred_splitk_fused_add_rms_norm_bit_exact(cuda, m, n, k):
    """linear(defer=True) -> fused_add_rms_norm reduces the split-K partials inside the norm
    kernel; it must equal reduce-then-norm bit for bit, and match the fp32 reference."""
    from distributed_llms_amd import ops
    from distributed_llms_amd.ops import gemm
    from distributed_llms_amd.ops import reference as ref
    torch.manual_seed(0)
    x = (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(n, device="cuda")).to(torch.bfloat16)
    res0 = torch.randn(m, n, device="cuda").to(torch.bfloat16)
    p = ops.linear(x, w, defer=True)
    assert isinstance(p, gemm.SplitKPartial) and p.splits > 1
    r1 = res0.clone()
    y1, _ = ops.fused_add_rms_norm(p, r1, g, 1e-5)
    p2 = ops.linear(x, w, defer=True)
    h = p2.materialize()
    r2 = res0.clone()
    y2, _ = ops.fused_add_rms_norm(h, r2, g, 1e-5)
    assert torch.equal(y1, y2) and torch.equal(r1, r2)
    torch.testing.assert_close(h.float(), ref.linear(x.float(), w.float()), atol=2e-2, rtol=2e-2)
    yr, rr = ref.fused_add_rms_norm(h.float(), res0.float(), g.float(), 1e-5)
    torch.testing.assert_close(y1.float(), yr, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [1, 100, 128, 129, 256, 384, 512])
@pytest.mark.parametrize("n,k,splits", [(6144, 4096, 1), (6144, 4096, 5), (4096, 14336, 8), (4096, 4096, 3),
                                        (1024, 512, 1)])
@pytest.mark.parametrize("variant", [0, 1])
def test_wide_linear(cuda, m, n, k, splits, variant):
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    y = gemm.linear_wide(x, w, splits=splits, variant=variant)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [7, 128, 256, 300])
@pytest.mark.parametrize("inter,k,splits", [(14336, 4096, 1), (1024, 512, 1), (1024, 1024, 2)])
@pytest.mark.parametrize("variant", [0, 1])
def test_wide_swiglu(cuda, m, inter, k, splits, variant):
    x, w = _bf(m, k), _bf(2 * inter, k, scale=0.05)
    y = gemm.linear_wide(x, w, splits=splits, swiglu=True, variant=variant)
    gu = x.float() @ w.float().t()
    ref = F.silu(gu[:, :inter]) * gu[:, inter:]
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [1, 37, 128, 200, 256, 300])
@pytest.mark.parametrize("n,k,splits,swiglu", [(6144, 4096, 5, False), (4096, 14336, 8, False),
                                               (1024, 512, 1, False), (2048, 512, 1, True)])
def test_wide_split_fragment_waits_bit_exact(cuda, m, n, k, splits, swiglu):
    """Variant bit 32 (fragment reads in asm, one lgkmcnt wait per MFMA row) runs the same MFMAs
    in the same order as the default K-tile: bit-identical outputs."""
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    a = gemm.linear_wide(x, w, splits=splits, swiglu=swiglu, variant=1)
    b = gemm.linear_wide(x, w, splits=splits, swiglu=swiglu, variant=1 | 32)
    assert torch.equal(a, b)


@pytest.mark.parametrize("m,n,k,splits,swiglu", [(256, 28672, 4096, 1, True), (256, 4096, 14336, 8, False),
                                                (256, 6144, 4096, 5, False), (192, 4096, 4096, 4, False),
                                                (128, 2048, 1024, 2, False), (40, 1024, 512, 1, False),
                                                (256, 2048, 192, 3, False), (64, 2048, 128, 2, True)])
def test_wide_l2_prefetch_bit_exact(cuda, m, n, k, splits, swiglu):
    """Variant bit 128 (one extra LDS-DMA per staging slot pulls a weight line PFD slots ahead into
    L2; counted waits move to G + 1) only changes timing: bit-identical to the same variant without
    it, for the unsplit SwiGLU grid (33), split-K grids (1), short K (fewer tiles than the prefetch
    distance) and the 64-row tile."""
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    for v in (1, 33):
        a = gemm.linear_wide(x, w, splits=splits, swiglu=swiglu, variant=v)
        b = gemm.linear_wide(x, w, splits=splits, swiglu=swiglu, variant=v | 128)
        assert torch.equal(a, b), v


@pytest.mark.parametrize("m,n,k,swiglu", [(4500, 1024, 512, False), (5000, 2048, 256, True), (2048, 256, 128, False)])
def test_wide_grouped_tile_order_bit_exact(cuda, m, n, k, swiglu):
    """Variant bit 64 (grouped row-tile order for prefill M) only reorders the workgroups: every
    tile runs the same MFMAs, so outputs are bit-identical to the plain order."""
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    a = gemm.linear_wide(x, w, splits=1, swiglu=swiglu, variant=4)
    b = gemm.linear_wide(x, w, splits=1, swiglu=swiglu, variant=4 | 64)
    assert torch.equal(a, b)
    ref = x.float() @ w.float().t()
    if swiglu:
        g, u = ref.chunk(2, -1)
        ref = torch.nn.functional.silu(g) * u
    torch.testing.assert_close(b.float(), ref, rtol=2e-2, atol=2e-2)


def test_splitk_slabs_keep_output_precision(cuda):
    """Split-K slabs are stored as f16 x 2^-6 (csrc/kernels/common.h, DLLM_PART_TYPE 2): the split
    result must stay within one bf16 ulp of the exact product (plus half an ulp of the output's typical
    magnitude, for outputs near zero), with a mean error no worse than 1.25x that of the unsplit
    kernel (whose only error is the bf16 output rounding)."""
    x, w = _bf(256, 14336), _bf(4096, 14336, scale=0.02)
    ref = x.float() @ w.float().t()
    e1 = (gemm.linear_wide(x, w, splits=1).float() - ref).abs()
    e8 = (gemm.linear_wide(x, w, splits=8).float() - ref).abs()
    assert e8.mean() <= 1.25 * e1.mean(), (e8.mean().item(), e1.mean().item())
    bound = ref.abs() * 2.0 ** -7 + ref.std() * 2.0 ** -8
    assert bool((e8 <= bound).all()), (e8 - bound).max().item()


def test_wide_deferred_splitk_matches_materialized(cuda):
    x, w = _bf(256, 14336), _bf(4096, 14336, scale=0.02)
    p = gemm.linear_wide(x, w, splits=8, defer=True)
    assert isinstance(p, gemm.SplitKPartial) and p.splits == 8
    y = p.materialize()
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("bm", [64, 128, 192])
@pytest.mark.parametrize("m", [100, 256, 384])
def test_wide_row_tile_override(cuda, bm, m):
    """gemm_wide with a forced smaller row tile (variant bits 8.., what knobs.wide_small_bm selects):
    several M tiles per N tile, plain and deferred split-K."""
    from distributed_llms_amd import _ext
    x, w = _bf(m, 4096), _bf(4096, 4096, scale=0.05)
    ref = x.float() @ w.float().t()
    y = torch.empty(m, 4096, dtype=torch.bfloat16, device="cuda")
    ws = gemm._workspace(x.device)
    stream = torch.cuda.current_stream().cuda_stream
    _ext.kernels().gemm_wide(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, 4096, 4096, 4,
                             0, 1 | (bm << 8), stream)
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    s = _ext.kernels().gemm_wide(0, x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, 4096, 4096, 4, 2,
                                 1 | (bm << 8), stream)
    p = gemm.SplitKPartial(ws, s, m, 4096, (m, 4096), x.dtype, x.device)
    torch.testing.assert_close(p.materialize().float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [640, 768])
def test_wide_linear_past_512_rows(cuda, m):
    """knobs.wide_down_max_m > 512 routes M > 512 down projections to gemm_wide: three 256-row
    tiles (the 192-row tile is only used up to 384) with an 8-way K split."""
    x, w = _bf(m, 14336), _bf(4096, 14336, scale=0.05)
    y = gemm.linear_wide(x, w, splits=8)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


def test_deferred_down_at_768_rows_into_fused_norm(cuda, monkeypatch):
    """ops.linear(defer=True) at M = 768 with the down cutover raised: the deferred split-K partial
    feeds fused_add_rms_norm and matches the fp32 reference."""
    from distributed_llms_amd.ops import reference as ref
    from distributed_llms_amd import knobs
    monkeypatch.setattr(knobs.K, "wide", "auto")
    monkeypatch.setattr(knobs.K, "wide_down_max_m", 768)
    torch.manual_seed(1)
    m, n, k = 768, 4096, 14336
    x = (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(n, device="cuda")).to(torch.bfloat16)
    res0 = torch.randn(m, n, device="cuda").to(torch.bfloat16)
    p = ops.linear(x, w, defer=True)
    assert isinstance(p, gemm.SplitKPartial) and p.splits > 1 and p.m == m
    r = res0.clone()
    y, _ = ops.fused_add_rms_norm(p, r, g, 1e-5)
    h = ref.linear(x.float(), w.float())
    yr, rr = ref.fused_add_rms_norm(h, res0.float(), g.float(), 1e-5)
    torch.testing.assert_close(r.float(), rr, atol=6e-2, rtol=3e-2)
    torch.testing.assert_close(y.float(), yr, atol=6e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [129, 200, 256])
@pytest.mark.parametrize("n,k,splits", [(6144, 4096, 0), (4096, 14336, 0), (4096, 4096, 16), (1024, 512, 1),
                                        (512, 1024, 3)])
def test_sq_linear(cuda, m, n, k, splits):
    """256 x 256-tile decode GEMM (gemm_sq.hip) vs fp32, split and unsplit, partial row tile."""
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    y = gemm.linear_sq(x, w, splits=splits)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [130, 256])
@pytest.mark.parametrize("inter,k,splits", [(14336, 4096, 0), (1024, 512, 1), (1024, 1024, 2)])
def test_sq_swiglu(cuda, m, inter, k, splits):
    """SwiGLU: fused epilogue (1 slice, interleaved gate / up rows) and split-K + SwiGLU reduce."""
    x, w = _bf(m, k), _bf(2 * inter, k, scale=0.05)
    y = gemm.linear_sq(x, w, splits=splits, swiglu=True)
    gu = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), F.silu(gu[:, :inter]) * gu[:, inter:], atol=3e-2, rtol=3e-2)


def test_sq_deferred_into_fused_norm(cuda):
    from distributed_llms_amd.ops import reference as ref
    torch.manual_seed(3)
    m, n, k = 256, 4096, 14336
    x = (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(n, device="cuda")).to(torch.bfloat16)
    res0 = torch.randn(m, n, device="cuda").to(torch.bfloat16)
    p = gemm.linear_sq(x, w, defer=True)
    assert isinstance(p, gemm.SplitKPartial) and p.splits == 16
    r = res0.clone()
    y, _ = ops.fused_add_rms_norm(p, r, g, 1e-5)
    yr, rr = ref.fused_add_rms_norm(ref.linear(x.float(), w.float()), res0.float(), g.float(), 1e-5)
    torch.testing.assert_close(r.float(), rr, atol=6e-2, rtol=3e-2)
    torch.testing.assert_close(y.float(), yr, atol=6e-2, rtol=3e-2)


# ---- gemm_pp: ping-pong 256-row-tile kernel (decode split-K, prefill grouped + SwiGLU)
@pytest.mark.parametrize("m", [1, 77, 200, 256, 300, 777])
@pytest.mark.parametrize("n,k,splits", [(6144, 4096, 1), (6144, 4096, 10), (4096, 14336, 16), (512, 192, 3),
                                        (512, 128, 2), (256, 320, 1)])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 4, 5, 64, 65, 66, 68, 69])
def test_pp_linear(cuda, m, n, k, splits, variant):
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    y = gemm.linear_pp(x, w, splits=splits, variant=variant)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [64, 256, 1000])
@pytest.mark.parametrize("inter,k,splits", [(14336, 4096, 1), (14336, 4096, 2), (384, 256, 1)])
@pytest.mark.parametrize("variant", [0, 1, 4, 5, 6, 64, 65, 68])
def test_pp_swiglu(cuda, m, inter, k, splits, variant):
    if variant & 1 == 0 and (2 * inter) % 256:
        pytest.skip("256-column tile needs 2I % 256 == 0")
    torch.manual_seed(m * 7 + splits + variant)
    x, w = _bf(m, k), _bf(2 * inter, k, scale=0.05)
    y = gemm.linear_pp(x, w, splits=splits, swiglu=True, variant=variant)
    gu = x.float() @ w.float().t()
    ref = F.silu(gu[:, :inter]) * gu[:, inter:]
    # gate and up pass through f16 split-K slabs (splits > 1) or bf16 (schedule 2's two-phase
    # epilogue) before the SiLU: absolute error up to ~(|u| + 1) x their rounding (|u| ~ 3 here)
    torch.testing.assert_close(y.float(), ref, atol=6e-2, rtol=3e-2)


# ---- gemm_pf: persistent schedule-2 prefill kernel (tiles per workgroup > 1, row tails, tiny grids)
@pytest.mark.parametrize("m", [1, 77, 256, 300, 2048, 4100, 9000])
@pytest.mark.parametrize("n,k", [(6144, 4096), (4096, 14336), (512, 192), (256, 64), (1024, 128)])
def test_pf_linear(cuda, m, n, k):
    torch.manual_seed(m + n + k)
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    y = gemm.linear_pf(x, w)
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [64, 1000, 4096])
@pytest.mark.parametrize("inter,k", [(14336, 4096), (384, 256), (128, 64)])
def test_pf_swiglu(cuda, m, inter, k):
    torch.manual_seed(m * 3 + inter)
    x, w = _bf(m, k), _bf(2 * inter, k, scale=0.05)
    y = gemm.linear_pf(x, w, swiglu=True)
    gu = x.float() @ w.float().t()
    ref = F.silu(gu[:, :inter]) * gu[:, inter:]
    torch.testing.assert_close(y.float(), ref, atol=6e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [256, 2100])
def test_pf_swiglu_nontemporal_stores_bit_exact(cuda, m):
    """SwiGLU with the nontemporal output stores (variant 8; the default above 256 MiB of output):
    the same bits as the default stores, rows past M dropped."""
    x, w = _bf(m, 1024), _bf(2 * 1536, 1024, scale=0.05)
    assert torch.equal(gemm.linear_pf(x, w, swiglu=True, variant=8), gemm.linear_pf(x, w, swiglu=True))


def test_pf_matches_pp_schedule2_bit_exact(cuda):
    """Same K-tile body and accumulation order as gemm_pp schedule 2: identical bits, plain and
    SwiGLU (the SwiGLU of gemm_pp rounds gate / up to bf16 first, so only the plain form is exact)."""
    x, w = _bf(5000, 4096), _bf(6144, 4096, scale=0.05)
    assert torch.equal(gemm.linear_pf(x, w), gemm.linear_pp(x, w, splits=1, variant=gemm.PP_PREFILL_VARIANT))


def test_pf_swiglu_output_range_is_the_half_width(cuda):
    """SwiGLU's output is [M, N / 2]: a 70B prefill gate|up (M 32768, 2I 57344) is within the
    kernel's 2 GiB output range although M x 2I x 2 bytes is not (a small-K stand-in shape)."""
    x, w = _bf(32768, 64), _bf(57344, 64, scale=0.05)
    y = gemm.linear_swiglu(x, w)
    assert y.shape == (32768, 28672)
    gu = x[-300:].float() @ w.float().t()
    ref = F.silu(gu[:, :28672]) * gu[:, 28672:]
    torch.testing.assert_close(y[-300:].float(), ref, atol=6e-2, rtol=3e-2)


def test_pf_dispatch_and_graph(cuda):
    from distributed_llms_amd import knobs
    x, w = _bf(4096, 4096), _bf(4096, 4096, scale=0.05)
    with knobs.override(pp_proj_min_m=2048, pp_persistent=True):
        y0 = gemm.linear(x, w)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = gemm.linear(x, w)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


def test_pp_deferred_splitk_matches_materialized_and_wide(cuda):
    x, w = _bf(256, 14336), _bf(4096, 14336, scale=0.05)
    p = gemm.linear_pp(x, w, splits=16, defer=True)
    assert isinstance(p, gemm.SplitKPartial) and p.splits == 16
    y = p.materialize()
    ref = x.float() @ w.float().t()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    # the slabs feed the fused add + RMSNorm exactly as gemm_wide's do
    res = _bf(256, 4096)
    g = _bf(4096)
    a, ra = ops.fused_add_rms_norm(gemm.linear_pp(x, w, splits=16, defer=True), res.clone(), g, 1e-5)
    b, rb = ops.fused_add_rms_norm(y, res.clone(), g, 1e-5)
    torch.testing.assert_close(ra.float(), rb.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(a.float(), b.float(), atol=3e-2, rtol=3e-2)


def test_pp_graph_replay_and_determinism(cuda):
    x, w = _bf(256, 4096), _bf(6144, 4096, scale=0.05)
    y0 = gemm.linear_pp(x, w, splits=10)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        y = gemm.linear_pp(x, w, splits=10)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(y, y0)


@pytest.mark.parametrize("m", [225, 256])
def test_long_k_down_on_split_gemm_pp(cuda, m):
    """knobs.pp_down_min_k: a long-K down projection (K >= the knob) at decode M on split gemm_pp
    128-column tiles with nontemporal weights -- direct and deferred (partials reduced by the
    consumer) against fp32."""
    x, w = _bf(m, 16384), _bf(2048, 16384, scale=0.02)
    ref = x.float() @ w.float().t()
    with gemm.knobs.override(pp_down_min_k=16384):
        y = gemm.linear(x, w)
        d = gemm.linear(x, w, defer=True)
        assert isinstance(d, gemm.SplitKPartial)
        d = d.materialize()
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(d.float(), ref, atol=3e-2, rtol=3e-2)
