"""Mixtral MoE on the GPU (route + grouped expert GEMMs + combine) vs the fp32 PyTorch reference."""
import pytest
import torch

from distributed_llms_amd import ops
from distributed_llms_amd.ops import moe
from distributed_llms_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _bf(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


@pytest.mark.parametrize("t", [1, 7, 64, 200, 300])
@pytest.mark.parametrize("e,k,h,i", [(8, 2, 512, 384), (4, 2, 256, 256), (8, 1, 256, 128)])
def test_moe_forward(cuda, t, e, k, h, i):
    x = _bf(t, h)
    wr = _bf(e, h, scale=0.1)
    wgu = _bf(e, 2 * i, h, scale=0.05)
    wd = _bf(e, h, i, scale=0.05)
    out = ops.moe_forward(x, wr, wgu, wd, k)
    # reference with the same bf16 router logits the GPU path routes on
    logits = ref.linear(x, wr).float()
    tw, tid = ref.moe_route(logits, k)
    expect = ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid)
    torch.testing.assert_close(out.float(), expect, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("t", [40, 100, 150])
def test_moe_skewed_routing_multi_chunk(cuda, t):
    """All tokens routed to the same two experts: far more rows per expert than the row tile the
    expected count selected (t*k/e -> 16/32/64-row tiles) exercises the row-chunk loop."""
    e, k, h, i = 8, 2, 256, 256
    x = _bf(t, h)
    wr = torch.zeros(e, h, device="cuda", dtype=torch.bfloat16)
    wr[3] = 0.05
    wr[5] = 0.04
    x = x.abs()                                   # positive rows -> experts 3 and 5 always win
    wgu, wd = _bf(e, 2 * i, h, scale=0.05), _bf(e, h, i, scale=0.05)
    out = moe.forward(x, wr, wgu, wd, k)
    tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
    assert set(tid.unique().tolist()) == {3, 5}
    expect = ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid)
    torch.testing.assert_close(out.float(), expect, atol=3e-2, rtol=3e-2)


def test_moe_graph_capturable(cuda):
    t, e, k, h, i = 32, 8, 2, 256, 256
    x, wr = _bf(t, h), _bf(e, h, scale=0.1)
    wgu, wd = _bf(e, 2 * i, h, scale=0.05), _bf(e, h, i, scale=0.05)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        moe.forward(x, wr, wgu, wd, k)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = moe.forward(x, wr, wgu, wd, k)
    for _ in range(2):
        x.copy_(_bf(t, h))
        g.replay()
        torch.cuda.synchronize()
        tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
        torch.testing.assert_close(out.float(), ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid),
                                   atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("t", [1, 7, 40, 64, 150, 256])
@pytest.mark.parametrize("skew", [False, True])
def test_moe_wide_grouped_kernel(cuda, monkeypatch, t, skew):
    """The MFMA-tiled grouped expert GEMM (gemm_wide.hip moe_wide_gemm) forced for every token
    count: 64-row tiles, 128-row chunks, multi-chunk experts (skewed routing) and empty experts."""
    from distributed_llms_amd import knobs
    monkeypatch.setattr(knobs.K, "moe_wide_min_pairs", 1)
    e, k, h, i = 8, 2, 512, 384
    x = _bf(t, h)
    if skew:
        x = x.abs()
        wr = torch.zeros(e, h, device="cuda", dtype=torch.bfloat16)
        wr[2] = 0.05
        wr[6] = 0.04
    else:
        wr = _bf(e, h, scale=0.1)
    wgu, wd = _bf(e, 2 * i, h, scale=0.05), _bf(e, h, i, scale=0.05)
    out = moe.forward(x, wr, wgu, wd, k)
    tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
    expect = ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid)
    torch.testing.assert_close(out.float(), expect, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("t,h,i", [(64, 128, 128), (150, 512, 384), (256, 1024, 2048), (40, 4096, 256)])
def test_moe_wide_deep_ring_bit_exact(cuda, monkeypatch, t, h, i):
    """The deep LDS ring of the grouped expert GEMM (6 / 5 slots) against the 3-slot ring: same
    K-tile order, so bit-identical outputs; K from 2 K-tiles (shorter than the ring) to 64."""
    from distributed_llms_amd import knobs
    monkeypatch.setattr(knobs.K, "moe_wide_min_pairs", 1)
    e, k = 8, 2
    x, wr = _bf(t, h), _bf(e, h, scale=0.1)
    wgu, wd = _bf(e, 2 * i, h, scale=0.05), _bf(e, h, i, scale=0.05)
    monkeypatch.setattr(knobs.K, "moe_deep_ring", True)
    deep = moe.forward(x, wr, wgu, wd, k)
    monkeypatch.setattr(knobs.K, "moe_deep_ring", False)
    shallow = moe.forward(x, wr, wgu, wd, k)
    assert torch.equal(deep, shallow)
    tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
    # the bf16 SwiGLU intermediate rounds at K = 4096: tolerance scaled to the output magnitude
    expect = ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid)
    torch.testing.assert_close(deep.float(), expect, atol=2e-2 * expect.abs().max().item(), rtol=3e-2)


@pytest.mark.parametrize("t", [1, 5, 64, 256])
@pytest.mark.parametrize("e", [8, 16])
def test_fused_router_matches_library_path(cuda, monkeypatch, t, e):
    """Fused router GEMV + top-k + scatter vs library router GEMM + route kernel: same experts and
    weights (logits rounded to bf16 in both), a consistent expert-sorted slot layout."""
    from distributed_llms_amd import _ext
    k_, h = 2, 4096
    x, wr = _bf(t, h), _bf(e, h, scale=0.05)
    kern = _ext.kernels()
    st = torch.cuda.current_stream().cuda_stream
    outs = []
    for fused in (True, False):
        tw = torch.empty(t, k_, dtype=torch.float32, device="cuda")
        tid = torch.empty(t, k_, dtype=torch.int32, device="cuda")
        cnt = torch.empty(e, dtype=torch.int32, device="cuda")
        off = torch.empty(e + 1, dtype=torch.int32, device="cuda")
        srt = torch.empty(t * k_, dtype=torch.int32, device="cuda")
        inv = torch.empty(t * k_, dtype=torch.int32, device="cuda")
        if fused:
            kern.moe_router_route(x.data_ptr(), wr.data_ptr(), t, h, e, k_, tw.data_ptr(), tid.data_ptr(),
                                  cnt.data_ptr(), off.data_ptr(), srt.data_ptr(), inv.data_ptr(), st)
        else:
            logits = ops.linear(x, wr)
            kern.moe_route(logits.data_ptr(), t, e, k_, tw.data_ptr(), tid.data_ptr(), cnt.data_ptr(),
                           off.data_ptr(), srt.data_ptr(), inv.data_ptr(), st)
        outs.append((tw, tid, cnt, off, srt, inv))
    (tw1, tid1, c1, o1, s1, i1), (tw2, tid2, c2, o2, s2, i2) = outs
    agree = (tid1 == tid2).all(dim=1)
    assert agree.float().mean() > 0.98                       # near-tie flips from accumulation order only
    # weights: one bf16 ulp of a logit (different accumulation order) moves a softmax weight ~1 %
    torch.testing.assert_close(tw1[agree], tw2[agree], atol=3e-2, rtol=3e-2)
    tok = torch.arange(t, device="cuda").repeat_interleave(k_)
    assert torch.equal(s1[i1.long()], tok.to(torch.int32))    # inv and sorted lists are consistent
    assert int(o1[-1]) == t * k_ and torch.equal(torch.diff(o1), c1)


@pytest.mark.parametrize("t,e,k,h,i,skew", [(4096, 8, 2, 1024, 2048, True), (4096, 8, 2, 1024, 2048, False),
                                            (777, 8, 2, 512, 384, True), (300, 4, 1, 256, 128, False),
                                            (4096, 8, 2, 4096, 14336, True)])
def test_moe_prefill_grouped_gemm(cuda, t, e, k, h, i, skew):
    """Prefill-sized T runs the device-side grouped GEMM (gemm_pp_moe: every expert's row tiles in
    one launch per projection, counts read on the device): skewed routing (two experts take most
    rows, the others few or none -> row tiles of many sizes, empty experts, tiles that end inside
    a segment) vs the fp32 reference on the same routing."""
    torch.manual_seed(t + h)
    x = _bf(t, h)
    if skew:
        x = x.abs() * 0.5
        wr = _bf(e, h, scale=0.002)
        wr[1] += 0.03
        wr[6] += 0.02
    else:
        wr = _bf(e, h, scale=0.1)
    wgu, wd = _bf(e, 2 * i, h, scale=0.03), _bf(e, h, i, scale=0.03)
    out = moe.forward(x, wr, wgu, wd, k)
    tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
    expect = ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid)
    tol = 2e-2 * expect.abs().max().item()
    torch.testing.assert_close(out.float(), expect, atol=tol, rtol=3e-2)


def test_moe_prefill_has_no_host_sync(cuda):
    """The prefill MoE path captures into a HIP graph (a host sync -- reading the expert counts on
    the host -- would fail the capture) and replays correctly for new inputs."""
    t, e, k, h, i = 2048, 8, 2, 512, 512
    x, wr = _bf(t, h), _bf(e, h, scale=0.1)
    wgu, wd = _bf(e, 2 * i, h, scale=0.05), _bf(e, h, i, scale=0.05)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        moe.forward(x, wr, wgu, wd, k)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = moe.forward(x, wr, wgu, wd, k)
    x.copy_(_bf(t, h))
    g.replay()
    torch.cuda.synchronize()
    tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
    expect = ref.moe_mlp(x.float(), wgu.float(), wd.float(), tw, tid)
    torch.testing.assert_close(out.float(), expect, atol=2e-2 * expect.abs().max().item(), rtol=3e-2)


def test_moe_fp8_prefill_grouped_no_host_sync(cuda):
    """W8A8 experts at prefill-sized T: one grouped fp8 launch per projection (no expert loop, no
    counts read on the host -- graph-capturable), against the fp8 reference numerics."""
    from distributed_llms_amd.ops import quant
    t, e, k, h, i = 1024, 8, 2, 512, 512
    torch.manual_seed(3)
    x, wr = _bf(t, h), _bf(e, h, scale=0.1)
    wgu, wd = quant.quantize_experts(_bf(e, 2 * i, h, scale=0.05)), quant.quantize_experts(_bf(e, h, i, scale=0.05))
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        moe.forward(x, wr, wgu, wd, k)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        out = moe.forward(x, wr, wgu, wd, k)
    g.replay()
    torch.cuda.synchronize()
    tw, tid = ref.moe_route(ref.linear(x, wr).float(), k)
    expect = quant.moe_mlp_ref(x, wgu, wd, tw, tid)
    torch.testing.assert_close(out.float(), expect.float(), atol=3e-2 * expect.abs().max().item(), rtol=5e-2)
