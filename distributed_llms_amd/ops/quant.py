"""FP8 (OCP e4m3) W8A8 decode GEMMs -- the quantization capability the reference only documents
(``plan.md:109-112,438-456``, ``snippets.md:684-833`` sketch bitsandbytes int8/int4
with an absmax fallback; the reference code never quantizes anything).

MI355X-native form: CDNA4's block-scaled MFMA (``v_mfma_scale_f32_16x16x128_f8f6f4``) runs e4m3 at
twice the bf16 rate, and an e4m3 weight is half the bytes, so the decode projections -- which sit on
the bf16 ridge at batch 256 -- get both halves of their bound cut:

* weights: per-output-channel absmax scales, quantized once at load (:func:`quantize_weight`);
* activations: per-token absmax scales, quantized on the fly by ``quant_fp8_rows``
  (csrc/kernels/quant.hip);
* GEMM: ``gemm_wide_fp8`` (csrc/kernels/gemm_wide.hip) -- the wide kernel's LDS-DMA pipeline with
  fp8 K-tiles of 128, scales applied in the epilogue (also before SwiGLU and before split-K slabs,
  so the bf16 path's deferred reductions are reused unchanged).

Mixtral experts take the same scheme through the grouped kernel (``moe_wide_gemm_fp8``: fp8 token
rows gathered by the expert-sorted slot list, per-(expert, channel) weight scales).

Opt-in (``EngineConfig.quant = "fp8"``, ``bench.py --quant fp8``): the LM head, embeddings, norms,
router, attention and the KV cache stay bf16.  CPU tensors take the PyTorch reference below (same
quantization, f32 math), which is also the numerics oracle of the GPU tests.
"""
from __future__ import annotations

from typing import Tuple

import torch

from .. import _ext, knobs

FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0
QUANT_KEYS = ("wqkv", "wo", "w_gate_up", "w_down")
EXPERT_KEYS = ("experts_gate_up", "experts_down")


class Fp8Weight:
    """An [N, K] weight as e4m3 values ``q`` and per-row (output channel) f32 ``scale``:
    w ~= q * scale[:, None]."""

    __slots__ = ("q", "scale")

    def __init__(self, q: torch.Tensor, scale: torch.Tensor):
        if q.dtype != FP8 or q.dim() != 2 or scale.shape != (q.shape[0],) or scale.dtype != torch.float32:
            raise ValueError("Fp8Weight: q [N, K] float8_e4m3fn and scale [N] float32")
        self.q, self.scale = q.contiguous(), scale.contiguous()

    @property
    def shape(self):
        return self.q.shape

    @property
    def device(self):
        return self.q.device

    @property
    def dtype(self):
        return FP8

    def numel(self) -> int:
        return self.q.numel()

    def nbytes(self) -> int:
        return self.q.numel() + 4 * self.scale.numel()

    def dequantize(self, dtype=torch.float32) -> torch.Tensor:
        return (self.q.float() * self.scale[:, None]).to(dtype)

    def __repr__(self):
        return f"Fp8Weight(shape={tuple(self.q.shape)}, device={self.q.device})"


class Fp8Experts:
    """A stack of expert weights [E, N, K] as e4m3 ``q`` with per-(expert, channel) f32 ``scale``
    [E, N]; ``experts[j]`` is expert j's :class:`Fp8Weight`."""

    __slots__ = ("q", "scale")

    def __init__(self, q: torch.Tensor, scale: torch.Tensor):
        if q.dtype != FP8 or q.dim() != 3 or scale.shape != q.shape[:2] or scale.dtype != torch.float32:
            raise ValueError("Fp8Experts: q [E, N, K] float8_e4m3fn and scale [E, N] float32")
        self.q, self.scale = q.contiguous(), scale.contiguous()

    @property
    def shape(self):
        return self.q.shape

    @property
    def device(self):
        return self.q.device

    @property
    def dtype(self):
        return FP8

    def is_contiguous(self) -> bool:
        return True

    def numel(self) -> int:
        return self.q.numel()

    def nbytes(self) -> int:
        return self.q.numel() + 4 * self.scale.numel()

    def __getitem__(self, j: int) -> Fp8Weight:
        return Fp8Weight(self.q[j], self.scale[j])

    def __repr__(self):
        return f"Fp8Experts(shape={tuple(self.q.shape)}, device={self.q.device})"


class Fp8Act:
    """A per-token quantized activation [..., K]: e4m3 ``q`` [M, K], f32 ``scale`` [M].  Produced by
    the norm kernels when the next GEMM takes fp8 (``ops.rms_norm(..., quant=True)``), consumed by
    :func:`linear_fp8` without a separate quantization launch."""

    __slots__ = ("q", "scale", "shape", "dtype")

    def __init__(self, q, scale, shape, dtype):
        self.q, self.scale, self.shape, self.dtype = q, scale, tuple(shape), dtype

    @property
    def device(self):
        return self.q.device

    @property
    def is_cuda(self):
        return self.q.is_cuda

    def dequantize(self) -> torch.Tensor:
        return (self.q.float() * self.scale[:, None]).to(self.dtype).reshape(self.shape)


def _absmax_scale(amax: torch.Tensor) -> torch.Tensor:
    # a tensor divisor: torch divides a GPU tensor by a Python scalar as a multiply by its
    # (inexact) reciprocal; the kernel, and the CPU, divide correctly rounded
    return torch.where(amax > 0, amax / torch.full_like(amax, FP8_MAX), torch.ones_like(amax))


def quantize_weight(w: torch.Tensor) -> Fp8Weight:
    """Per-output-channel absmax quantization of an [N, K] weight (any float dtype, any device)."""
    wf = w.float()
    s = _absmax_scale(wf.abs().amax(dim=1))
    q = (wf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return Fp8Weight(q, s)


def quantize_experts(w: torch.Tensor) -> Fp8Experts:
    """Per-(expert, output channel) absmax quantization of an [E, N, K] expert stack."""
    wf = w.float()
    s = _absmax_scale(wf.abs().amax(dim=2))
    q = (wf / s[..., None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return Fp8Experts(q, s)


def quantize_rows_ref(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-row (per-token) absmax quantization, PyTorch reference: (q [M, K] e4m3, scale [M] f32)."""
    xf = x.reshape(-1, x.shape[-1]).float()
    s = _absmax_scale(xf.abs().amax(dim=1))
    return (xf / s[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8), s


def quantize_rows(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-token quantization of a bf16 activation [..., K] -> (q [M, K] e4m3, scale [M] f32); the
    HIP kernel on the GPU (bit-identical to :func:`quantize_rows_ref`)."""
    if not x.is_cuda:
        return quantize_rows_ref(x)
    if x.dtype != torch.bfloat16 or not x.is_contiguous():
        raise ValueError("quantize_rows: bf16 contiguous activations")
    k = x.shape[-1]
    m = x.numel() // k
    if k % 8:
        raise ValueError("quantize_rows: K % 8")
    q = torch.empty(m, k, dtype=FP8, device=x.device)
    s = torch.empty(m, dtype=torch.float32, device=x.device)
    _ext.kernels().quant_fp8_rows(q.data_ptr(), s.data_ptr(), x.data_ptr(), m, k,
                                  torch.cuda.current_stream().cuda_stream)
    return q, s


def linear_ref(x, w: Fp8Weight, swiglu: bool = False) -> torch.Tensor:
    """The W8A8 product in f32 from the quantized operands (CPU path and GPU-test oracle);
    ``x``: a float tensor (quantized here) or an :class:`Fp8Act`."""
    q, s = (x.q, x.scale) if isinstance(x, Fp8Act) else quantize_rows_ref(x)
    y = (q.float() * s[:, None]) @ w.dequantize(torch.float32).t().to(q.device)
    if swiglu:
        g, u = y.chunk(2, dim=-1)
        y = torch.nn.functional.silu(g) * u
    return y.to(x.dtype).reshape(*x.shape[:-1], y.shape[-1])


# 128 < M <= 256 split-K grids (qkv / o / down): two 128-row tiles with at most half the K slices
# instead of one 256-row tile -- a third fewer staged bytes per workgroup per K-tile (the loop is
# bound by its LDS-DMA staging).  bench/fp8_bench.py --sweep at M = 256 (us, default 1-tile plan ->
# this): o_8b 21.4 -> 18.0, qkv_8b 20.3 -> 19.1 (2 slices; 3 slices: 26.0), down_8b 29.3 = 29.3
# (knobs.fp8_bm128)
# prefill-sized M (no K split): grouped row-tile order (gemm_wide_fp8 variant bit 64) from this M:
# at M = 32768 qkv 1018 -> 889 us, o 660 -> 599, gate|up 4509 -> 3924, down 2083 -> 1873 (1.8-2.0
# PFLOP/s); at M = 2048 it is 1-6 % slower
# PFLOP/s); at M = 2048 it is 1-6 % slower (knobs.fp8_group_m)


def fp8_plan(m: int, n: int, k: int, swiglu: bool = False) -> Tuple[int, int]:
    """(K slices, row-tile override or 0) of gemm_wide_fp8 for this shape.  Default: the bf16
    kernel's rule on the 128-K tiles (a K-tile of fp8 holds the bytes of a 64-K bf16 tile)."""
    from .gemm import wide_splits
    s = wide_splits(m, n, k // 2, swiglu)
    if knobs.K.fp8_bm128 and not swiglu and s > 1 and 128 < m <= 256:
        tiles = (n // 128) * 2
        return max(1, min(256 // tiles, (k // 128) // 4, 16)), 128
    return s, 0


def fp8_splits(m: int, n: int, k: int, swiglu: bool = False) -> int:
    return fp8_plan(m, n, k, swiglu)[0]


def linear_fp8(x: torch.Tensor, w: Fp8Weight, swiglu: bool = False, defer: bool = False, splits: int = 0):
    """y = x w^T (``swiglu``: silu(x Wg^T) * (x Wu^T), w = [Wg; Wu]) with W8A8 e4m3 operands.
    ``defer``: may return a :class:`~distributed_llms_amd.ops.gemm.SplitKPartial` (no SwiGLU)."""
    if not x.is_cuda:
        return linear_ref(x, w, swiglu)
    from .gemm import SplitKPartial, _workspace
    pre = isinstance(x, Fp8Act)
    k = x.shape[-1]
    n, kw = w.shape
    if kw != k:
        raise ValueError(f"linear_fp8: x[..., {k}] vs w {tuple(w.shape)}")
    if n % 128 or k % 128:
        raise ValueError("linear_fp8: N % 128 and K % 128")
    if x.dtype != torch.bfloat16:
        raise TypeError("linear_fp8: bf16 activations")
    if pre:
        xq, xs = x.q, x.scale
        m = xq.shape[0]
    else:
        x = x.contiguous()
        m = x.numel() // k
        xq, xs = quantize_rows(x)
    s, bm = fp8_plan(m, n, k, swiglu)
    if splits:
        s, bm = splits, 0
    ws = _workspace(x.device)
    if s > 1 and s * m * n > ws.numel():
        s = max(1, ws.numel() // (m * n))
    # weights streamed non-temporal only where one row tile covers M (each weight byte read once)
    variant = (1 if m <= 256 else (4 | (64 if 0 < knobs.K.fp8_group_m <= m else 0))) | (bm << 8)
    stream = torch.cuda.current_stream().cuda_stream
    kern = _ext.kernels()
    if defer and not swiglu and s > 1:
        se = kern.gemm_wide_fp8(0, xq.data_ptr(), xs.data_ptr(), w.q.data_ptr(), w.scale.data_ptr(), ws.data_ptr(),
                                ws.numel(), m, n, k, s, 2, variant, stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    kern.gemm_wide_fp8(y.data_ptr(), xq.data_ptr(), xs.data_ptr(), w.q.data_ptr(), w.scale.data_ptr(), ws.data_ptr(),
                       ws.numel(), m, n, k, s, 1 if swiglu else 0, variant, stream)
    return y


def moe_mlp_ref(x: torch.Tensor, w_gate_up: Fp8Experts, w_down: Fp8Experts, topk_w: torch.Tensor,
                topk_ids: torch.Tensor) -> torch.Tensor:
    """Mixtral expert MLPs with W8A8 experts (reference): per-token e4m3 inputs, per-row e4m3
    SwiGLU outputs, f32 products -- the numerics of the grouped fp8 kernels."""
    t, h = x.shape
    out = torch.zeros(t, h, dtype=torch.float32, device=x.device)
    for e in range(w_gate_up.shape[0]):
        tok, slot = (topk_ids == e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        y = linear_ref(linear_ref(x[tok], w_gate_up[e], swiglu=True), w_down[e])
        out.index_add_(0, tok, y.float() * topk_w[tok, slot].unsqueeze(1).float())
    return out.to(x.dtype)


def quantize_layers(layers, keys=QUANT_KEYS, expert_keys=EXPERT_KEYS) -> int:
    """Replace the dense projections (and MoE expert stacks) of every layer dict by
    :class:`Fp8Weight` / :class:`Fp8Experts` (in place); returns how many were converted.  The
    router, norms and biases stay as they are."""
    def ok(t, dims):
        # the GPU kernels tile N and K by 128 (CPU reference: any shape)
        return isinstance(t, torch.Tensor) and t.dim() == dims and (
            not t.is_cuda or (t.shape[-2] % 128 == 0 and t.shape[-1] % 128 == 0))
    n = 0
    for lw in layers:
        for name in keys:
            if ok(lw.get(name), 2):
                lw[name] = quantize_weight(lw[name])
                n += 1
        for name in expert_keys:
            if ok(lw.get(name), 3):
                lw[name] = quantize_experts(lw[name])
                n += 1
    return n
