"""Dense GEMM dispatch for y = x @ w^T (w is [N, K], nn.Linear layout).

Decode-sized M goes to hand-written gfx950 kernels, per projection role (cutovers measured in
the engine on Llama-3-8B, profiles/wide_gemm.md; each one is a field of :mod:`..knobs`):

* wide-M kernel (gemm_wide.hip: 64/128/192/256-row x 128 tiles, 3-stage LDS-DMA pipeline,
  split-K over workgroups) for every decode M:
  - gate|up (SwiGLU fused into the epilogue): M <= knobs.wide_gate_up_max_m (256);
  - down (K >= 8192 and K > N; split-K partials deferred into the next norm):
    M <= knobs.wide_down_max_m (512);
  - the other projections (qkv, o, LM head): M <= knobs.wide_proj_max_m (256); the o-projection
    (N K <= knobs.wide_small_bm_maxw) on 128-row tiles with half the K slices (knobs.wide_small_bm);
  with the 256 x 256 tile (gemm_sq.hip) taking unsplit grids at 225 <= M <= 256 (70B gate|up);
* the decode LM head at 225 <= M <= 256: gemm_pp.hip schedule 2 with nontemporal weights
  (knobs.pp_head_min_m);
* the decode SwiGLU gate|up at 200 <= M <= 256 on gemm_pp unsplit with nontemporal weights, on the
  column tile (128, else 256) that makes one round of CUs / 2 .. CUs tiles (8B: 224 x 128, 70B:
  224 x 256; knobs.pp_gate_up_min_m), and the long-K down projection (K >= knobs.pp_down_min_k,
  70B) at 225 <= M <= 256 on split gemm_pp 128-column tiles (profiles/round6_gate_up_pp.md);
* prefill (M >= knobs.pp_swiglu_min_m / pp_proj_min_m, above the decode ranges): the 4-wave
  256 x 256-tile schedule-2 kernel in its persistent form (gemm_pf in gemm_pp.hip, knobs.pp_persistent)
  -- gate|up with the SwiGLU fused into its epilogue, qkv / o / down plain
  (profiles/round4_gemm_counters.md);
* what none of them takes (a bias, N not a multiple of 256, fp32 on CPU, operands >= 4 GiB):
  torch's F.linear.

The role is inferred from the shape: "down" = K >= 8192 and K > N, so the square / widening
K = 8192 projections of 70B-class models (qkv 8192 -> 10240, o 8192 -> 8192) stay "proj".
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn.functional as F

from .. import _ext
from .. import knobs


def is_down_proj(n: int, k: int) -> bool:
    """The MLP down projection's shape: long, narrowing K (8B: 14336 -> 4096, 70B: 28672 -> 8192).
    A K = 8192 qkv or o projection of a 70B-class model (N >= K) is not one."""
    return k >= 8192 and k > n


def _cus(device) -> int:
    if torch.device(device).type != "cuda":
        return 256                     # MI355X (dispatch unit tests on CPU)
    idx = device.index or 0
    n = _CUS.get(idx)
    if n is None:
        n = _CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return n


_CUS = {}


def pf_fills(m: int, n: int, device) -> bool:
    """gemm_pf (one 256 x 256 tile per CU per round, no split-K) only where its grid fills the chip:
    at least one tile per CU and rounds that are mostly full (knobs.pf_min_eff), or many rounds.
    Below that the split-K gemm_pp grid wins at every measured M from 320 to 2048 -- gemm_pf's
    single-round grids run one tile's whole K loop: 74-78 us for the 8B o-projection at any
    M <= 2048, the down projection 250-283 us vs 55-174 us split (profiles/round5_medium_m_gemm.md)."""
    cus = _cus(device)
    tiles = (-(-m // 256)) * (n // 256)
    if tiles < cus:
        return False
    rounds = -(-tiles // cus)
    return rounds >= 4 or tiles / (rounds * cus) >= knobs.K.pf_min_eff


def _use_wide(m: int, n: int, k: int, x: torch.Tensor, w: torch.Tensor, swiglu: bool = False) -> bool:
    kn = knobs.K
    roles = {t for t in kn.wide.split(",") if t and t != "none"}
    if not roles or m < 1 or n % 128 or k % 64:
        return False
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        return False
    down = is_down_proj(n, k) and not swiglu
    if "all" in roles:
        return m <= 512 or (down and m <= kn.wide_down_max_m)
    if "auto" in roles:
        if swiglu:
            return m <= kn.wide_gate_up_max_m
        if down:
            return m <= kn.wide_down_max_m
        return m <= (kn.wide_o_max_m if n <= k else kn.wide_proj_max_m)
    if swiglu:
        return "gate_up" in roles and m <= 512
    return ("down" in roles) if is_down_proj(n, k) else ("proj" in roles and m <= 512)


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


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, defer: bool = False):
    """y = x w^T (+bias).  ``defer``: may return a :class:`SplitKPartial` (see there)."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if w.shape[1] != k:
        raise ValueError(f"linear: x[..., {k}] vs w {tuple(w.shape)}")
    kn = knobs.K
    # decode LM head on gemm_pp with nontemporal weights (236 vs 268 us for gemm_sq at M = 256) --
    # unless comm kernels may hold CUs: beside a 4-workgroup, 20 KiB-LDS receive spinning in
    # another process it took 284 us, gemm_sq 268 either way (bench/debug/lm_head_bench.py,
    # profiles/round5_raw/r5ae_head.txt) -- the pipeline's last stage holds the head
    if bias is None and n > 65536 and 0 < kn.pp_head_min_m <= m <= 256 \
            and (not _comm_cus or kn.head_beside_comm == "pp") and _use_pp(m, n, k, x, w, 1):
        return linear_pp(x, w, splits=1, variant=PP_HEAD_VARIANT)           # decode LM head
    if bias is None and 0 < kn.pp_down_min_k <= k and 225 <= m <= 256 and is_down_proj(n, k) and not _comm_cus \
            and n % 128 == 0 and _use_pp(m, n, k, x, w, 1):
        # long-K decode down projection (70B: K = 28672) on gemm_pp's 128-column tile, K slices filling
        # the CUs, weights nontemporal: 126 vs 135 us for gemm_wide (bench/debug/medium_m_sweep.py)
        s = max(1, min(16, _cus(x.device) // (n // 128)))
        return linear_pp(x, w, splits=s, defer=defer, variant=64 | 2 | 1)
    if bias is None and _use_wide(m, n, k, x, w):
        return linear_wide(x, w, defer=defer)
    if bias is None and _use_pp(m, n, k, x, w, knobs.K.pp_proj_min_m):
        if kn.pp_persistent and m * n * 2 < (1 << 31) and pf_fills(m, n, x.device):
            return linear_pf(x, w)
        # medium M (mixed prefill + decode steps, short prompts): split-K tiles fill the CUs
        return linear_pp(x, w, variant=PP_PREFILL_VARIANT, defer=defer)
    return F.linear(x, w, bias)


PP_PREFILL_VARIANT = 64 | 4        # gemm_pp: schedule 2, grouped row-tile order, 256-column tile
PP_GATE_UP_VARIANT = 64 | 2 | 1    # gemm_pp: schedule 2, nontemporal weights, 128-column tile
PP_HEAD_VARIANT = 64 | 2           # gemm_pp: schedule 2, nontemporal weights (read once per step)


def _use_pp(m: int, n: int, k: int, x: torch.Tensor, w: torch.Tensor, min_m: int) -> bool:
    """Prefill-sized GEMM on gemm_pp (knobs.pp_swiglu_min_m / pp_proj_min_m)."""
    return (0 < min_m <= m and n % 256 == 0 and k % 64 == 0 and x.dtype == w.dtype == torch.bfloat16
            and x.is_contiguous() and w.is_contiguous() and m * k * 2 < (1 << 32) and n * k * 2 < (1 << 32))


_ws = {}
_WS_FLOATS = 32 << 20          # 128 MiB of split-K partials per (device, stream)


def _workspace(device: torch.device) -> torch.Tensor:
    key = (device.index or 0, torch.cuda.current_stream().cuda_stream)
    t = _ws.get(key)
    if t is None:
        t = _ws[key] = torch.empty(_WS_FLOATS, dtype=torch.float32, device=device)
    return t


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


def wide_row_tile(m: int, n: int, k: int, swiglu: bool = False) -> int:
    """Row tile gemm_wide uses for this shape (knobs.wide_small_bm for small split grids, else
    wide_bm): e.g. 128 runs an M = 256 o-projection as 2 row tiles x 4 K slices instead of 1 x 8."""
    kn = knobs.K
    if kn.wide_small_bm and not swiglu and n * k <= kn.wide_small_bm_maxw and kn.wide_small_bm < wide_bm(m):
        return kn.wide_small_bm
    return wide_bm(m)


# CUs a co-resident communication kernel may hold (set by the RCCL transport of a pipeline stage:
# a p2p receive spins on its CUs for as long as its peer has not sent).  gemm_wide's split-K grids
# are sized to leave them free: its workgroups (144 KiB of LDS) cannot share a CU with a kernel
# holding LDS, so a 256-workgroup grid beside 4 such CUs runs a second round for 4 workgroups --
# the down projection took 1.58x its solo time beside a 4-CU receive, the 224 / 240-workgroup
# grids 1.00x (scripts/hwq_probe.py gemms, profiles/round5_comm_queues.md)
_comm_cus = 0
_comm_users = 0


def pf_dynamic() -> bool:
    """gemm_pf's dynamic tile queue: knobs.pf_dynamic "on" / "off" / "auto" (on while comm kernels
    may hold CUs)."""
    v = str(knobs.K.pf_dynamic).strip().lower()
    if v == "auto":
        return _comm_cus > 0
    return v in ("1", "true", "on", "yes")


def reserve_cus_for_comm(n: int) -> None:
    """A transport with spinning comm kernels starts: size gemm_wide grids around ``n`` CUs."""
    global _comm_cus, _comm_users
    _comm_users += 1
    _comm_cus = max(_comm_cus, int(n))


def release_cus_for_comm() -> None:
    global _comm_cus, _comm_users
    _comm_users = max(0, _comm_users - 1)
    if not _comm_users:
        _comm_cus = 0


def wide_splits(m: int, n: int, k: int, swiglu: bool = False, target_wgs: int = 0) -> int:
    """K slices for gemm_wide: about one workgroup per CU, >= 8 K-tiles (512) per slice (with CUs
    reserved for communication: at most one workgroup per remaining CU)."""
    tiles = (n // 128) * (-(-m // wide_row_tile(m, n, k, swiglu)))
    target = target_wgs or knobs.K.wide_target_wgs
    if _comm_cus:
        s = max(1, (target - _comm_cus) // tiles)
    else:
        s = max(1, round(target / tiles))
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
    v = (knobs.K.wide_variant_split if s > 1 else knobs.K.wide_variant) if variant < 0 else variant
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


def linear_pf(x: torch.Tensor, w: torch.Tensor, swiglu: bool = False, variant: int = 0) -> torch.Tensor:
    """Persistent prefill GEMM (gemm_pf in csrc/kernels/gemm_pp.hip): schedule 2's 256 x 256 tiles,
    one workgroup per CU walking its tiles with the LDS-DMA pipeline running across tile
    boundaries; optional fused SwiGLU (``w`` = [Wg; Wu], y [M, N / 2]).  ``variant`` 8: nontemporal
    output stores (the default for SwiGLU outputs > 256 MiB); the tiles come from per-XCD device
    queues while knobs.pf_dynamic says so (bit 16 of the launcher's variant)."""
    k = x.shape[-1]
    n = w.shape[0]
    m = x.numel() // k
    if not (x.dtype == w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()):
        raise ValueError("linear_pf: bf16 contiguous operands")
    if n % 256 or k % 64:
        raise ValueError("linear_pf: N % 256 and K % 64")
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    dyn = pf_dynamic() and k >= 128
    if torch.cuda.is_current_stream_capturing():
        # inside a graph: the static tile walk.  A tile queue is per stream and self-resetting, but
        # a replay may run on another stream beside eager launches that use the same queue
        dyn = False
    if dyn:
        variant |= 16                  # per-XCD dynamic tile queues (gemm_pp.hip, DYN)
    _ext.kernels().gemm_pf(y.data_ptr(), x.data_ptr(), w.data_ptr(), m, n, k, 1 if swiglu else 0, variant,
                           torch.cuda.current_stream().cuda_stream)
    return y


# 256 x 256-tile decode GEMM (gemm_sq.hip) for 128 < M <= 256: a third fewer staged bytes per FLOP
# than the wide kernel's 256 x 128 tile.  Measured (profiles/wide_gemm.md, "256 x 256 tile"): it
# wins only where the grid needs no K split -- the LM head (1.05x) and the 70B MLP gate|up (1.07x);
# split grids (8B qkv / o / gate|up / down) lose 6-20 % to the extra slab traffic.  knobs.sq: roles
# (gate_up, down, proj, head, all) or none; knobs.sq_split also admits split grids; knobs.sq_min_m
# (225: at M = 192 it loses 1-6 %).


def sq_role(n: int, k: int, swiglu: bool) -> str:
    if swiglu:
        return "gate_up"
    if is_down_proj(n, k):
        return "down"
    return "head" if n > 65536 else "proj"


def use_sq(m: int, n: int, k: int, swiglu: bool = False) -> bool:
    kn = knobs.K
    roles = {t for t in kn.sq.split(",") if t and t != "none"}
    if not roles or not (kn.sq_min_m <= m <= 256) or n % 256 or k % 64:
        return False
    if not kn.sq_split and sq_splits(m, n, k) > 1:
        return False
    return "all" in roles or sq_role(n, k, swiglu) in roles


def sq_splits(m: int, n: int, k: int, target_wgs: int = 256) -> int:
    """K slices for gemm_sq: as many as keep (N / 256) x slices within one workgroup per CU, at
    least 4 K-tiles (256) per slice."""
    tiles = (n // 256) * (-(-m // 256))
    return max(1, min(target_wgs // max(1, tiles), (k // 64) // 4, 16))


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
    v = knobs.K.sq_variant if variant < 0 else variant
    if defer and not swiglu and s > 1:
        se = _ext.kernels().gemm_sq(0, x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s, 2, v,
                                    stream)
        return SplitKPartial(ws, se, m, n, (*x.shape[:-1], n), x.dtype, x.device)
    y = torch.empty(*x.shape[:-1], n // 2 if swiglu else n, dtype=x.dtype, device=x.device)
    _ext.kernels().gemm_sq(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, n, k, s,
                           1 if swiglu else 0, v, stream)
    return y


def linear_swiglu(x: torch.Tensor, w_gate_up: torch.Tensor) -> Optional[torch.Tensor]:
    """silu(x Wg^T) * (x Wu^T) with W = [Wg; Wu] in one launch; None if the shape is not eligible."""
    k = x.shape[-1]
    n = w_gate_up.shape[0]
    m = x.numel() // k
    kn = knobs.K
    if 0 < kn.pp_gate_up_min_m <= m <= 256 and not _comm_cus and _use_pp(m, n, k, x, w_gate_up, 1):
        # decode gate|up on gemm_pp, unsplit, weights nontemporal, on the column tile that gives one
        # round of CUs / 2 .. CUs tiles: 8B (224 x 128 columns) 62.1 vs 64.1 us for gemm_wide, 70B
        # (224 x 256 columns) 204 vs 259 us for gemm_sq (bench/debug/medium_m_sweep.py --pp)
        cus = _cus(x.device)
        if n % 128 == 0 and cus // 2 <= n // 128 <= cus:
            return linear_pp(x, w_gate_up, splits=1, swiglu=True, variant=PP_GATE_UP_VARIANT)
        if n % 256 == 0 and cus // 2 <= n // 256 <= cus:
            return linear_pp(x, w_gate_up, splits=1, swiglu=True, variant=PP_GATE_UP_VARIANT & ~1)
    if _use_wide(m, n, k, x, w_gate_up, swiglu=True):
        return linear_wide(x, w_gate_up, swiglu=True)
    if _use_pp(m, n, k, x, w_gate_up, knobs.K.pp_swiglu_min_m):
        if knobs.K.pp_persistent and m * (n // 2) * 2 < (1 << 31) and pf_fills(m, n, x.device):
            return linear_pf(x, w_gate_up, swiglu=True)
        return linear_pp(x, w_gate_up, swiglu=True, variant=PP_PREFILL_VARIANT)
    return None
