"""Dense GEMM dispatch for y = x @ w^T (w is [N, K], nn.Linear layout).

Decode-sized M goes to hand-written gfx950 kernels, per projection role (cutovers measured in
the engine on Llama-3-8B, profiles/wide_gemm.md; each one is an environment knob):

* wide-M kernel (gemm_wide.hip: 64/128/192/256-row x 128 tiles, 3-stage LDS-DMA pipeline):
  - gate|up (SwiGLU fused into the epilogue): M <= 256 (DLLM_WIDE_GATE_UP_MAX_M);
  - down (K >= 8192 and K > N; split-K partials deferred into the next norm): M <= 512
    (DLLM_WIDE_DOWN_MAX_M, may be raised past 512);
  - the other projections (qkv, o, LM head): M <= 256 (DLLM_WIDE_PROJ_MAX_M);
* tiny M outside those (DLLM_WIDE off): weight-streaming MFMA GEMV (gemm_skinny.hip);
* 64 <= M <= 512 with K >= 8192 when the wide kernel is off: split-K LDS-tiled MFMA kernel
  (gemm_tiled.hip);
* everything else (prefill, M above the cutovers): hipBLASLt via torch (TunableOp table in
  tuning/), the only non-HIP GPU path, chosen purely by shape.

The role is inferred from the shape: "down" = K >= 8192 and K > N, so the square / widening
K = 8192 projections of 70B-class models (qkv 8192 -> 10240, o 8192 -> 8192) stay "proj".
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.nn.functional as F

from .. import _ext

SKINNY_MAX_M = 64
# Engine dispatch: the weight-streaming kernel serves M <= engine_skinny_max_m(N, K).  Measured
# against hipBLASLt with cold caches (bench/gemm_bench.py, profiles/gemm_skinny_v3_vs_hipblaslt.txt):
# with the coalesced k-permutation it streams 4-5 TB/s at M <= 4 and wins 1.4-1.8x on the MLP and
# big projections, less as M grows; the LM head (N > 64K) stays on hipBLASLt (4.6 TB/s there).
SKINNY_ENABLED = os.environ.get("DLLM_SKINNY", "1") != "0"


def engine_skinny_max_m(n: int, k: int) -> int:
    if not SKINNY_ENABLED or n > 65536:
        return 0
    # in-engine A/B (warm, TunableOp-tuned hipBLASLt, HIP graphs; scripts/gpu_ab_skinny.sh):
    # B=1 +6.6 %, B=8/16 -1..-4 % with the cold-cache thresholds (16/8/2) -> keep it to M <= 4
    e = n * k
    if e >= 50_000_000:       # 8B gate|up (117M) and down (59M), 70B qkv / down / gate|up
        return 4
    if e >= 16_000_000:       # 8B o (17M), 8B qkv (25M)
        return 2
    return 0


def skinny_ok(m: int, n: int, k: int, x: torch.Tensor, w: torch.Tensor, swiglu: bool = False,
              force: bool = False) -> bool:
    lim = SKINNY_MAX_M if force else engine_skinny_max_m(n, k)
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and 1 <= m <= lim
            and k % 128 == 0 and n % (32 if swiglu else 16) == 0 and x.is_contiguous() and w.is_contiguous())


def _launch(x, w, bias, y, m, n, k, mode):
    _ext.kernels().gemm_skinny(y.data_ptr(), x.data_ptr(), w.data_ptr(), 0 if bias is None else bias.data_ptr(),
                               m, n, k, mode, torch.cuda.current_stream().cuda_stream)


# Which GEMM serves decode-sized M (64 <= M <= 512):
#   DLLM_GEMM=auto  (default) tiled split-K kernel for long-K projections (K >= 8192: the MLP down
#                   projection), where it measured 1.24-2.0x hipBLASLt (profiles/gemm_tiled_vs_hipblaslt.txt);
#                   hipBLASLt elsewhere (ties or wins there)
#   DLLM_GEMM=tiled / blas  force one implementation (A/B experiments)
GEMM_MODE = os.environ.get("DLLM_GEMM", "auto")
#   DLLM_TILED_NMAX=<n>: (auto mode) also route shapes with N <= n to the tiled kernel (A/B knob)
TILED_NMAX = int(os.environ.get("DLLM_TILED_NMAX", "0"))


def _use_tiled(m: int, n: int, k: int, x: torch.Tensor, w: torch.Tensor) -> bool:
    if GEMM_MODE == "blas" or not (64 <= m <= 512) or n % 128 or k % 64:
        return False
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        return False
    return GEMM_MODE == "tiled" or k >= 8192 or n <= TILED_NMAX


# DLLM_WIDE: which decode-sized (M <= 512) GEMMs the wide-M kernel (gemm_wide.hip) serves:
#   comma list of gate_up (SwiGLU-fused MLP up projection), down (K >= 8192, deferred split-K),
#   proj (the other projections: qkv, o), all, or none.  Default "auto", from the in-engine A/B
#   (scripts/gpu_ab_wide.sh, profiles/wide_gemm.md): gate_up + down for M <= 512 (+4.3 % at
#   B=256, +5.8 % at B=128, +1.2 % at B=512), proj only up to M = 256 (it loses at 512), gate_up
#   only up to M = 256 (DLLM_WIDE_GATE_UP_MAX_M: hipBLASLt + silu_mul is +1.9 % at B=384, +2.5 % at 512).
WIDE = {t for t in os.environ.get("DLLM_WIDE", "auto").split(",") if t and t != "none"}
# gemm_wide variant: 1 = LDS-DMA pieces interleaved with the MFMAs (weights nt where the grid has no
# K split); | 32 = fragment reads in asm with one lgkmcnt wait per MFMA row instead of hipcc's
# lgkmcnt(0) before a K-tile's first MFMA (bit-exact).  In-engine (profiles/wide_gemm.md) bit 32
# speeds up the unsplit SwiGLU gate|up grid (68.7 -> 66.9 us at B = 256) and slows the split-K
# qkv / o / down grids (24.7 -> 26.3 us), so split grids keep variant 1: Llama-3-8B B = 256
# 27,014 (all 1) / 26,896 (all 33) / 27,123 tok/s (this split), interleaved on one box.
WIDE_VARIANT = int(os.environ.get("DLLM_WIDE_VARIANT", "33"))
# variant for split-K grids (qkv / o / down at decode M)
WIDE_VARIANT_SPLIT = int(os.environ.get("DLLM_WIDE_VARIANT_SPLIT", "1"))


# smallest M the wide kernel serves (1: every decode batch; the 64-row tile at M <= 64 streams
# the weights at 4.5-6.4 TB/s, +15-19 % tok/s over skinny / hipBLASLt at B = 1..64)
WIDE_MIN_M = int(os.environ.get("DLLM_WIDE_MIN_M", "1"))
# largest M the SwiGLU-fused gate|up projection runs on the wide kernel under "auto" (above it:
# hipBLASLt + silu_mul); profiles/wide_gemm.md "gate|up tile / split / cutover"
WIDE_GATE_UP_MAX_M = int(os.environ.get("DLLM_WIDE_GATE_UP_MAX_M", "256"))
# same for the K >= 8192 (MLP down) projection, whose split-K output defers into the next norm
WIDE_DOWN_MAX_M = int(os.environ.get("DLLM_WIDE_DOWN_MAX_M", "512"))
# and for the other projections (qkv, o)
WIDE_PROJ_MAX_M = int(os.environ.get("DLLM_WIDE_PROJ_MAX_M", "256"))


def is_down_proj(n: int, k: int) -> bool:
    """The MLP down projection's shape: long, narrowing K (8B: 14336 -> 4096, 70B: 28672 -> 8192).
    A K = 8192 qkv or o projection of a 70B-class model (N >= K) is not one."""
    return k >= 8192 and k > n


def _use_wide(m: int, n: int, k: int, x: torch.Tensor, w: torch.Tensor, swiglu: bool = False) -> bool:
    if not WIDE or GEMM_MODE == "blas" or not (WIDE_MIN_M <= m <= max(512, WIDE_DOWN_MAX_M)) or n % 128 or k % 64:
        return False
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        return False
    if "all" in WIDE:
        return m <= 512 or (is_down_proj(n, k) and not swiglu and m <= WIDE_DOWN_MAX_M)
    if "auto" in WIDE:
        if swiglu:
            return m <= WIDE_GATE_UP_MAX_M
        return m <= (WIDE_DOWN_MAX_M if is_down_proj(n, k) else WIDE_PROJ_MAX_M)
    if swiglu:
        return "gate_up" in WIDE and m <= 512
    return ("down" in WIDE) if is_down_proj(n, k) else ("proj" in WIDE and m <= 512)


class SplitKPartial:
    """Split-K partial sums of ``x @ w.T`` still in the per-stream workspace (not reduced).  Each K
    slice accumulates in f32; the slabs hold it as f16 x 2^-6 by default (csrc/kernels/common.h
    ``DLLM_PART_TYPE``: half the bytes of f32 slabs, 3 significand bits more than the bf16 result).

    Returned by ``linear(..., defer=True)`` when the split-K tiled kernel ran, so the NEXT op can
    fuse the reduction (``ops.fused_add_rms_norm`` -> splitk_add_rms_norm); anything else calls
    :meth:`materialize`.  Valid only until the next tiled GEMM on the same stream reuses the
    workspace -- consume it immediately."""

    __slots__ = ("ws", "splits", "m", "n", "shape", "dtype", "device")

    def __init__(self, ws, splits, m, n, shape, dtype, device):
        self.ws, self.splits, self.m, self.n = ws, splits, m, n
        self.shape, self.dtype, self.device = shape, dtype, device

    def materialize(self) -> torch.Tensor:
        y = torch.empty(self.shape, dtype=self.dtype, device=self.device)
        _ext.kernels().splitk_reduce(y.data_ptr(), self.ws.data_ptr(), 0, self.splits, self.m, self.n,
                                     torch.cuda.current_stream().cuda_stream)
        return y


def _effective_splits(k: int, splits: int) -> int:
    kps = -(-(k // 64) // splits) * 64            # same rounding as csrc/kernels/gemm_tiled.hip
    return -(-k // kps)


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           force_skinny: bool = False, defer: bool = False):
    """y = x w^T (+bias).  ``defer``: may return a :class:`SplitKPartial` (see there)."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if w.shape[1] != k:
        raise ValueError(f"linear: x[..., {k}] vs w {tuple(w.shape)}")
    # the wide kernel first: with its 64-row tile it streams the weights faster than the skinny
    # kernel and hipBLASLt at every decode M (profiles/wide_gemm.md, "small M")
    if bias is None and not force_skinny and _use_wide(m, n, k, x, w):
        return linear_wide(x, w, defer=defer)
    if skinny_ok(m, n, k, x, w, force=force_skinny) and (bias is None or bias.dtype == torch.bfloat16):
        y = torch.empty(*x.shape[:-1], n, dtype=x.dtype, device=x.device)
        _launch(x, w, bias, y, m, n, k, 0)
        return y
    if _use_tiled(m, n, k, x, w) and (bias is None or bias.dtype == torch.bfloat16):
        if defer and bias is None:
            return linear_tiled(x, w, None, defer=True)
        return linear_tiled(x, w, bias)
    return F.linear(x, w, bias)


_ws = {}
_WS_FLOATS = 32 << 20          # 128 MiB of split-K partials per (device, stream)


def _workspace(device: torch.device) -> torch.Tensor:
    key = (device.index or 0, torch.cuda.current_stream().cuda_stream)
    t = _ws.get(key)
    if t is None:
        t = _ws[key] = torch.empty(_WS_FLOATS, dtype=torch.float32, device=device)
    return t


def tiled_splits(m: int, n: int, k: int, target_wgs: int = 512) -> int:
    tiles = (n // 128) * (-(-m // 128))
    s = max(1, -(-target_wgs // tiles))
    return max(1, min(s, k // 512, 16))


def linear_tiled(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, splits: int = 0,
                 swiglu: bool = False, defer: bool = False):
    """Split-K LDS-tiled MFMA GEMM (csrc/kernels/gemm_tiled.hip) for decode-sized M."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        raise ValueError("linear_tiled: bf16 contiguous operands")
    if n % 128 or k % 64:
        raise ValueError("linear_tiled: N % 128 and K % 64")
    s = splits or tiled_splits(m, n, k)
    ncols = n // 2 if swiglu else n
    y = torch.empty(*x.shape[:-1], ncols, dtype=x.dtype, device=x.device)
    ws = _workspace(x.device)
    if s * m * n > ws.numel():
        s = max(1, ws.numel() // (m * n))
    if defer and not swiglu and bias is None and _effective_splits(k, s) > 1:
        se = _effective_splits(k, s)
        _ext.kernels().gemm_tiled(0, x.data_ptr(), w.data_ptr(), 0, ws.data_ptr(), ws.numel(), m, n, k, s, 2,
                                  torch.cuda.current_stream().cuda_stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    _ext.kernels().gemm_tiled(y.data_ptr(), x.data_ptr(), w.data_ptr(), 0 if bias is None else bias.data_ptr(),
                              ws.data_ptr(), ws.numel(), m, n, k, s, 1 if swiglu else 0,
                              torch.cuda.current_stream().cuda_stream)
    return y


WIDE_TARGET_WGS = int(os.environ.get("DLLM_WIDE_TARGET", "256"))


def wide_bm(m: int) -> int:
    """Row tile of gemm_wide for M rows (mirrors wide_bm in csrc/kernels/gemm_wide.hip)."""
    if m <= 64:
        return 64
    if m <= 128:
        return 128
    if m <= 192:
        return 192
    if m <= 256:
        return 256
    return 192 if m <= 384 else 256


# Row tile override for split-K (non-SwiGLU) wide GEMMs with at most WIDE_SMALL_BM_MAXW weight
# elements: e.g. DLLM_WIDE_SMALL_BM=128 runs an M = 256 o-projection as 2 row tiles x 4 K slices
# instead of 1 x 8 (half the split-K slab bytes, 2/3 of the per-CU staging bytes per K-tile).
WIDE_SMALL_BM = int(os.environ.get("DLLM_WIDE_SMALL_BM", "0"))
WIDE_SMALL_BM_MAXW = int(os.environ.get("DLLM_WIDE_SMALL_BM_MAXW", str(4096 * 4096)))


def wide_row_tile(m: int, n: int, k: int, swiglu: bool = False) -> int:
    """Row tile gemm_wide uses for this shape (the override, else wide_bm)."""
    if WIDE_SMALL_BM and not swiglu and n * k <= WIDE_SMALL_BM_MAXW and WIDE_SMALL_BM < wide_bm(m):
        return WIDE_SMALL_BM
    return wide_bm(m)


def wide_splits(m: int, n: int, k: int, swiglu: bool = False, target_wgs: int = 0) -> int:
    """K slices for gemm_wide: about one workgroup per CU, >= 8 K-tiles (512) per slice."""
    tiles = (n // 128) * (-(-m // wide_row_tile(m, n, k, swiglu)))
    s = max(1, round((target_wgs or WIDE_TARGET_WGS) / tiles))
    return max(1, min(s, (k // 64) // 8, 16))


def linear_wide(x: torch.Tensor, w: torch.Tensor, splits: int = 0, swiglu: bool = False, defer: bool = False,
                variant: int = -1):
    """Wide-M decode GEMM (csrc/kernels/gemm_wide.hip): 256 x 128 x 64 tiles, 3-deep LDS-DMA pipeline,
    optional split-K and fused SwiGLU epilogue (``w`` = [Wg; Wu]).  ``defer``: may return a
    :class:`SplitKPartial` (no SwiGLU)."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if splits == 0 and variant < 0 and use_sq(m, n, k, swiglu):
        return linear_sq(x, w, swiglu=swiglu, defer=defer)
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        raise ValueError("linear_wide: bf16 contiguous operands")
    if n % 128 or k % 64:
        raise ValueError("linear_wide: N % 128 and K % 64")
    s = splits or wide_splits(m, n, k, swiglu)
    ws = _workspace(x.device)
    if s > 1 and s * m * n > ws.numel():
        s = max(1, ws.numel() // (m * n))
    stream = torch.cuda.current_stream().cuda_stream
    v = (WIDE_VARIANT_SPLIT if s > 1 else WIDE_VARIANT) if variant < 0 else variant
    bm = wide_row_tile(m, n, k, swiglu)
    if bm != wide_bm(m):
        v |= bm << 8
    if defer and not swiglu and s > 1:
        se = _ext.kernels().gemm_wide(0, x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s, 2, v, stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    _ext.kernels().gemm_wide(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s,
                             1 if swiglu else 0, v, stream)
    return y


def linear_big(x: torch.Tensor, w: torch.Tensor, splits: int = 2, swiglu: bool = False, defer: bool = False):
    """Experimental 256 x 256 x 32 tile with one 128 x 128 wave per SIMD (csrc/kernels/gemm_big.hip);
    split-K only for SwiGLU / deferred outputs."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        raise ValueError("linear_big: bf16 contiguous operands")
    ws = _workspace(x.device)
    stream = torch.cuda.current_stream().cuda_stream
    if defer and not swiglu and splits > 1:
        se = _ext.kernels().gemm_big(0, x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, splits, 2, stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    _ext.kernels().gemm_big(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, splits,
                            1 if swiglu else 0, stream)
    return y


def pp_splits(m: int, n: int, k: int, bn: int = 256, target_wgs: int = 256) -> int:
    """K slices for gemm_pp: about one workgroup per CU (tiles x slices <= target), >= 3 K-tiles
    (192) per slice."""
    tiles = (n // bn) * (-(-m // 256))
    return max(1, min(target_wgs // max(1, tiles), (k // 64) // 3, 32))


def linear_pp(x: torch.Tensor, w: torch.Tensor, splits: int = 0, swiglu: bool = False, defer: bool = False,
              variant: int = 0):
    """Ping-pong 256-row-tile GEMM (csrc/kernels/gemm_pp.hip).  ``variant``: bit 0 = 128-column tile
    (else 256), bit 1 = weights nontemporal, bit 2 = grouped row-tile order (large M).  Split-K
    partials are reduced by splitk_reduce(_swiglu), or returned as a :class:`SplitKPartial` with
    ``defer`` (no SwiGLU)."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        raise ValueError("linear_pp: bf16 contiguous operands")
    bn = 128 if variant & 1 else 256
    if n % bn or k % 64:
        raise ValueError(f"linear_pp: N % {bn} and K % 64")
    s = splits or pp_splits(m, n, k, bn)
    ws = _workspace(x.device)
    if s > 1 and s * m * n > ws.numel():
        s = max(1, ws.numel() // (m * n))
    stream = torch.cuda.current_stream().cuda_stream
    if defer and not swiglu and s > 1:
        se = _ext.kernels().gemm_pp(0, x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s, 2, variant,
                                    stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    _ext.kernels().gemm_pp(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s,
                           1 if swiglu else 0, variant, stream)
    return y


# 256 x 256-tile decode GEMM (gemm_sq.hip) for 128 < M <= 256: a third fewer staged bytes per FLOP
# than the wide kernel's 256 x 128 tile.  Measured (profiles/wide_gemm.md, "256 x 256 tile"): it
# wins only where the grid needs no K split -- the LM head (1.05x) and the 70B MLP gate|up (1.07x);
# split grids (8B qkv / o / gate|up / down) lose 6-20 % to the extra slab traffic.  DLLM_SQ: comma
# list of roles (gate_up, down, proj, head, all) or none; DLLM_SQ_SPLIT=1 also admits split grids.
SQ = {t for t in os.environ.get("DLLM_SQ", "all").split(",") if t and t != "none"}
SQ_MIN_M = int(os.environ.get("DLLM_SQ_MIN_M", "225"))   # at M = 192 it loses 1-6 %
SQ_SPLIT = os.environ.get("DLLM_SQ_SPLIT", "0") == "1"


def sq_role(n: int, k: int, swiglu: bool) -> str:
    if swiglu:
        return "gate_up"
    if is_down_proj(n, k):
        return "down"
    return "head" if n > 65536 else "proj"


def use_sq(m: int, n: int, k: int, swiglu: bool = False) -> bool:
    if not SQ or not (SQ_MIN_M <= m <= 256) or n % 256 or k % 64:
        return False
    if not SQ_SPLIT and sq_splits(m, n, k) > 1:
        return False
    return "all" in SQ or sq_role(n, k, swiglu) in SQ


def sq_splits(m: int, n: int, k: int, target_wgs: int = 256) -> int:
    """K slices for gemm_sq: as many as keep (N / 256) x slices within one workgroup per CU, at
    least 4 K-tiles (256) per slice."""
    tiles = (n // 256) * (-(-m // 256))
    return max(1, min(target_wgs // max(1, tiles), (k // 64) // 4, 16))


SQ_VARIANT = int(os.environ.get("DLLM_SQ_VARIANT", "4"))


def linear_sq(x: torch.Tensor, w: torch.Tensor, splits: int = 0, swiglu: bool = False, defer: bool = False,
              variant: int = -1):
    """256 x 256-tile decode GEMM (csrc/kernels/gemm_sq.hip); split-K partials reduced by
    splitk_reduce(_swiglu), or returned as a :class:`SplitKPartial` with ``defer`` (no SwiGLU)."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        raise ValueError("linear_sq: bf16 contiguous operands")
    if n % 256 or k % 64:
        raise ValueError("linear_sq: N % 256 and K % 64")
    s = splits or sq_splits(m, n, k)
    ws = _workspace(x.device)
    if s > 1 and s * m * n > ws.numel():
        s = max(1, ws.numel() // (m * n))
    stream = torch.cuda.current_stream().cuda_stream
    v = SQ_VARIANT if variant < 0 else variant
    if defer and not swiglu and s > 1:
        se = _ext.kernels().gemm_sq(0, x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s, 2, v,
                                    stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    _ext.kernels().gemm_sq(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s,
                           1 if swiglu else 0, v, stream)
    return y


def linear_swiglu(x: torch.Tensor, w_gate_up: torch.Tensor, force_skinny: bool = False) -> Optional[torch.Tensor]:
    """silu(x Wg^T) * (x Wu^T) with W = [Wg; Wu] in one launch; None if the shape is not eligible."""
    k = x.shape[-1]
    n = w_gate_up.shape[0]
    m = x.numel() // k
    if not force_skinny and _use_wide(m, n, k, x, w_gate_up, swiglu=True):
        return linear_wide(x, w_gate_up, swiglu=True)
    if not skinny_ok(m, n, k, x, w_gate_up, swiglu=True, force=force_skinny):
        return None
    y = torch.empty(*x.shape[:-1], n // 2, dtype=x.dtype, device=x.device)
    _launch(x, w_gate_up, None, y, m, n, k, 1)
    return y
