"""gemm_rw (register-weight decode GEMM, csrc/kernels/gemm_rw.hip) vs a plain fp32 PyTorch GEMM of
the same operands: plain / split-K / deferred slabs / fused SwiGLU, every ring depth, M tails."""
import pytest
import torch
import torch.nn.functional as F

from distributed_llms_amd import ops
from distributed_llms_amd.ops import gemm

pytestmark = pytest.mark.gpu


def _bf(*s, scale=1.0):
    return (torch.randn(*s, device="cuda") * scale).to(torch.bfloat16)


# ring depths each row tile is built with (csrc/kernels/gemm_rw.hip gemm_rw)
NS_OF = {256: (3, 4, 5), 128: (4, 6, 8), 64: (4, 8)}


def _ns(m, i):
    bm = 64 if m <= 64 else 128 if m <= 128 else 256
    if i >= len(NS_OF[bm]):
        pytest.skip(f"{bm}-row tile has {len(NS_OF[bm])} ring depths")
    return NS_OF[bm][i]


@pytest.mark.parametrize("m", [1, 31, 64, 100, 128, 255, 256])
@pytest.mark.parametrize("n,k,splits", [(6144, 4096, 1), (6144, 4096, 5), (4096, 14336, 8), (4096, 4096, 8),
                                        (1024, 512, 1), (256, 64, 1), (384, 192, 2)])
@pytest.mark.parametrize("nsi", [0, 1, 2])
def test_rw_linear(cuda, m, n, k, splits, nsi):
    ns = _ns(m, nsi)
    torch.manual_seed(m * 7 + n + k + ns)
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    y = gemm.linear_rw(x, w, splits=splits, variant=ns)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [1, 77, 256])
@pytest.mark.parametrize("inter,k,splits", [(14336, 4096, 1), (1024, 512, 1), (1024, 1024, 2), (64, 64, 1)])
@pytest.mark.parametrize("nsi", [0, 1, 2])
def test_rw_swiglu(cuda, m, inter, k, splits, nsi):
    ns = _ns(m, nsi)
    torch.manual_seed(m + inter + k + ns)
    x, w = _bf(m, k), _bf(2 * inter, k, scale=0.05)
    y = gemm.linear_rw(x, w, splits=splits, swiglu=True, variant=ns)
    gu = x.float() @ w.float().t()
    ref = F.silu(gu[:, :inter]) * gu[:, inter:]
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m", [1, 100, 256])
@pytest.mark.parametrize("n,k,splits,swiglu", [(6144, 4096, 5, False), (4096, 14336, 8, False), (28672, 4096, 1, True),
                                               (1024, 512, 1, True), (384, 192, 2, False), (1024, 1024, 2, True)])
@pytest.mark.parametrize("nsi", [0, 1])
def test_rw_packed_bit_exact(cuda, m, n, k, splits, swiglu, nsi):
    """Fragment-major packed weights (gemm.pack_rw) give the same bits as the nn.Linear layout:
    the same fragments in the same registers, only the load addresses differ."""
    ns = _ns(m, nsi)
    torch.manual_seed(m + n + k + ns)
    x, w = _bf(m, k), _bf(n, k, scale=0.05)
    a = gemm.linear_rw(x, w, splits=splits, swiglu=swiglu, variant=ns)
    b = gemm.linear_rw(x, gemm.pack_rw(w, swiglu), splits=splits, swiglu=swiglu, variant=ns, packed=True)
    assert torch.equal(a, b)
    if not swiglu:
        torch.testing.assert_close(b.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("m,n,k", [(256, 4096, 14336), (200, 4096, 4096), (64, 1024, 8192)])
def test_rw_deferred_splitk_fused_add_rms_norm(cuda, m, n, k):
    """Deferred split-K slabs reduced inside the next add + RMSNorm equal reduce-then-norm."""
    from distributed_llms_amd.ops import reference as ref
    torch.manual_seed(1)
    x = (torch.randn(m, k, device="cuda") * 0.5).to(torch.bfloat16)
    w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
    g = (1 + 0.1 * torch.randn(n, device="cuda")).to(torch.bfloat16)
    res0 = torch.randn(m, n, device="cuda").to(torch.bfloat16)
    p = gemm.linear_rw(x, w, defer=True)
    assert isinstance(p, gemm.SplitKPartial) and p.splits > 1
    r1 = res0.clone()
    y1, _ = ops.fused_add_rms_norm(p, r1, g, 1e-5)
    h = gemm.linear_rw(x, w, defer=True).materialize()
    r2 = res0.clone()
    y2, _ = ops.fused_add_rms_norm(h, r2, g, 1e-5)
    assert torch.equal(y1, y2) and torch.equal(r1, r2)
    torch.testing.assert_close(h.float(), ref.linear(x.float(), w.float()), atol=2e-2, rtol=2e-2)


def test_rw_graph_replay(cuda):
    x, w = _bf(256, 4096), _bf(28672, 4096, scale=0.05)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gemm.linear_rw(x, w, swiglu=True)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        y = gemm.linear_rw(x, w, swiglu=True)
    for _ in range(3):
        x.copy_(_bf(256, 4096))
        g.replay()
        gu = x.float() @ w.float().t()
        torch.testing.assert_close(y.float(), F.silu(gu[:, :14336]) * gu[:, 14336:], atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("bm", [1, 2, 3])
def test_rw_row_tile_override(cuda, bm):
    """variant bits 8-9 force the 64 / 128 / 256-row tile for an M that fits it: same results."""
    x, w = _bf(50, 4096), _bf(4096, 4096, scale=0.05)
    y = gemm.linear_rw(x, w, splits=8, variant=bm << 8)
    torch.testing.assert_close(y.float(), x.float() @ w.float().t(), atol=3e-2, rtol=3e-2)


def test_rw_rejects_bad_shapes(cuda):
    with pytest.raises(ValueError):
        gemm.linear_rw(_bf(257, 256), _bf(256, 256))
    with pytest.raises(ValueError):
        gemm.linear_rw(_bf(8, 256), _bf(200, 256))
