"""Mixtral MoE: router (K11) and expert MLPs (K12).

GPU path (bf16):
  router logits  = linear(x, W_router)                                   [T, E]
  moe_route      : softmax -> top-k -> renormalise, expert-sorted slots    (HIP, one launch)
  decode-sized T : grouped weight-streaming GEMMs on the sorted slots (gate|up + SwiGLU, then down)
                   entirely on device -- no host sync, so the decode step stays graph-capturable
  prefill-sized T: grouped 256 x 256-tile GEMMs over the expert-sorted slots (gemm_pp.hip
                   gemm_pp_moe: one launch per projection, every expert's row tiles in one grid,
                   counts / offsets read on the device -- no host sync, no per-expert loop; gate|up
                   with the SwiGLU in its epilogue, the token gather in its A staging)
  W8A8 experts   : the grouped fp8 kernel (moe_wide_gemm_fp8) at every T, also without a host sync
  moe_combine    : weighted sum of each token's top-k expert outputs        (HIP)
CPU path: the PyTorch reference (ops/reference.py).
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from .. import _ext, knobs
from . import reference as ref

GROUPED_MAX_TOKENS = 256      # beyond this the per-expert row count makes library GEMMs cheaper
# knobs.moe_variant: 0 = pick by expected rows per expert; 1..6 force a kernel variant
# (bench/moe_bench.py sweeps them).  knobs.moe_wide_min_pairs: token-expert pairs (T x top_k) from
# which the MFMA-tiled grouped kernel (gemm_wide.hip moe_wide_gemm) replaces the weight-streaming
# one (moe.hip); 0 disables it.  Mixtral-8x7B end to end (in-engine A/B,
# profiles/moe_wide.md): B=1 0.95x, B=4 1.10x, B=16 1.10x, B=64 1.25x, B=128 1.52x, B=256 2.23x.
# knobs.moe_fused_router: decode router as fused GEMV + top-k + scatter kernels instead of library
# GEMM + route kernel.


def route(router_logits: torch.Tensor, top_k: int):
    return ref.moe_route(router_logits, top_k)


def mlp(x, w_gate_up, w_down, topk_w, topk_ids):
    return ref.moe_mlp(x, w_gate_up, w_down, topk_w, topk_ids)


def forward(x: torch.Tensor, w_router: torch.Tensor, w_gate_up: torch.Tensor, w_down: torch.Tensor,
            top_k: int, expert_offset: int = 0) -> torch.Tensor:
    """``w_gate_up`` / ``w_down`` may hold a contiguous range of the experts (expert parallelism):
    experts ``[expert_offset, expert_offset + w_gate_up.shape[0])`` of the router's E.  Routing is
    always over all E; tokens routed elsewhere contribute zero here, so the expert-parallel
    group's sum (an all-reduce) is the full MoE output."""
    e_all = w_router.shape[0]
    if not (0 <= expert_offset and expert_offset + w_gate_up.shape[0] <= e_all):
        raise ValueError(f"experts [{expert_offset}, {expert_offset + w_gate_up.shape[0]}) outside the router's {e_all}")
    from . import quant
    fp8 = isinstance(w_gate_up, quant.Fp8Experts)
    if fp8 != isinstance(w_down, quant.Fp8Experts):
        raise TypeError("moe: gate|up and down experts must both be fp8 or both not")
    if not x.is_cuda:
        tw, tid = ref.moe_route(ref.linear(x, w_router), top_k)
        if fp8:
            return quant.moe_mlp_ref(x, w_gate_up, w_down, tw, tid - expert_offset)
        return ref.moe_mlp(x, w_gate_up, w_down, tw, tid - expert_offset)
    from . import linear, linear_swiglu
    k = _ext.kernels()
    st = torch.cuda.current_stream().cuda_stream
    t, h = x.shape
    e_loc, two_i, _ = w_gate_up.shape
    e = e_all
    ep = e_loc != e_all
    inter = two_i // 2
    if not (x.is_contiguous() and w_gate_up.is_contiguous() and w_down.is_contiguous()):
        raise ValueError("moe: operands must be contiguous")
    dev = x.device
    topk_w = torch.empty(t, top_k, dtype=torch.float32, device=dev)
    topk_ids = torch.empty(t, top_k, dtype=torch.int32, device=dev)
    counts = torch.empty(e, dtype=torch.int32, device=dev)
    offsets = torch.empty(e + 1, dtype=torch.int32, device=dev)
    sorted_tok = torch.empty(t * top_k, dtype=torch.int32, device=dev)
    inv = torch.empty(t * top_k, dtype=torch.int32, device=dev)
    if knobs.K.moe_fused_router and e in (8, 16) and h % 32 == 0 and x.dtype == w_router.dtype == torch.bfloat16 \
            and w_router.is_contiguous():
        # router GEMV + softmax/top-k + scatter in two launches (no [T, E] logits round trip), at
        # decode and prefill T alike
        k.moe_router_route(x.data_ptr(), w_router.data_ptr(), t, h, e, top_k, topk_w.data_ptr(), topk_ids.data_ptr(),
                           counts.data_ptr(), offsets.data_ptr(), sorted_tok.data_ptr(), inv.data_ptr(), st)
    else:
        logits = linear(x, w_router)
        k.moe_route(logits.data_ptr(), t, e, top_k, topk_w.data_ptr(), topk_ids.data_ptr(), counts.data_ptr(),
                    offsets.data_ptr(), sorted_tok.data_ptr(), inv.data_ptr(), st)
    # expert parallel: only this rank's experts fill their slot rows; the others stay zero
    ys = (torch.zeros if ep else torch.empty)(t * top_k, h, dtype=x.dtype, device=dev)
    # the local experts' counts / offsets are a contiguous slice of the routing arrays
    cnt_p, off_p = counts.data_ptr() + 4 * expert_offset, offsets.data_ptr() + 4 * expert_offset
    if fp8:
        # W8A8 experts (ops/quant.py): per-token e4m3 x gathered by the grouped kernel (its scales in
        # slot order), SwiGLU output re-quantized per slot row for the down projection
        if x.dtype != torch.bfloat16 or two_i % 128 or h % 128 or inter % 128:
            raise ValueError("moe fp8: bf16 activations, expert dims multiples of 128")
        # one grouped launch per projection at every T (decode and prefill): each workgroup walks its
        # expert's row chunks for one column tile, counts / offsets read on the device -- no host
        # sync, no per-expert loop (round-4 review: the prefill used to loop over experts on the host)
        xq, xsc = quant.quantize_rows(x)
        sa = xsc.index_select(0, sorted_tok.long())
        act = torch.empty(t * top_k, inter, dtype=x.dtype, device=dev)
        k.moe_wide_gemm_fp8(act.data_ptr(), xq.data_ptr(), sorted_tok.data_ptr(), w_gate_up.q.data_ptr(), cnt_p,
                            off_p, e_loc, two_i, h, 1, sa.data_ptr(), w_gate_up.scale.data_ptr(), st)
        aq, asc = quant.quantize_rows(act)
        k.moe_wide_gemm_fp8(ys.data_ptr(), aq.data_ptr(), 0, w_down.q.data_ptr(), cnt_p, off_p, e_loc, h, inter,
                            0, asc.data_ptr(), w_down.scale.data_ptr(), st)
    elif t <= GROUPED_MAX_TOKENS:
        act = torch.empty(t * top_k, inter, dtype=x.dtype, device=dev)
        rows = -(-t * top_k // e)        # expected rows per expert picks the kernel's row tile
        if 0 < knobs.K.moe_wide_min_pairs <= t * top_k and x.dtype == torch.bfloat16 and two_i % 128 == 0 and h % 128 == 0 \
                and h % 64 == 0 and inter % 64 == 0:
            ring = 0 if knobs.K.moe_deep_ring else 4          # mode bit 2: the 3-slot LDS ring
            k.moe_wide_gemm(act.data_ptr(), x.data_ptr(), sorted_tok.data_ptr(), w_gate_up.data_ptr(),
                            cnt_p, off_p, e_loc, two_i, h, 1 | ring, st)
            k.moe_wide_gemm(ys.data_ptr(), act.data_ptr(), 0, w_down.data_ptr(), cnt_p, off_p, e_loc, h, inter,
                            ring, st)
        else:
            k.moe_grouped_gemm(act.data_ptr(), x.data_ptr(), sorted_tok.data_ptr(), w_gate_up.data_ptr(),
                               cnt_p, off_p, e_loc, two_i, h, 1, rows, knobs.K.moe_variant, st)
            k.moe_grouped_gemm(ys.data_ptr(), act.data_ptr(), 0, w_down.data_ptr(), cnt_p, off_p, e_loc, h, inter, 0,
                               rows, knobs.K.moe_variant, st)
    elif x.dtype == torch.bfloat16 and two_i % 256 == 0 and h % 256 == 0 and inter % 64 == 0 and h % 64 == 0 \
            and t * h * 2 < (1 << 32) and t * top_k * inter * 2 < (1 << 32):
        # prefill: one grouped launch per projection over every local expert's row tiles (the kernel
        # addresses each A operand with 32-bit buffer offsets: larger batches take the per-expert path)
        slots = t * top_k
        act = torch.empty(slots, inter, dtype=x.dtype, device=dev)
        k.gemm_pp_moe(act.data_ptr(), x.data_ptr(), sorted_tok.data_ptr(), w_gate_up.data_ptr(), cnt_p, off_p,
                      e_loc, two_i, h, t, slots, 1, st)
        k.gemm_pp_moe(ys.data_ptr(), act.data_ptr(), 0, w_down.data_ptr(), cnt_p, off_p, e_loc, h, inter, slots,
                      slots, 0, st)
    else:
        # odd expert dims (test-size models): per-expert GEMMs, counts read on the host
        xs = x.index_select(0, sorted_tok.long())
        off = offsets.cpu().tolist()
        for j in range(e_loc):
            a, b = off[expert_offset + j], off[expert_offset + j + 1]
            if b > a:
                ys[a:b] = F.linear(linear_swiglu(xs[a:b], w_gate_up[j]), w_down[j])
    out = torch.empty_like(x)
    k.moe_combine(out.data_ptr(), ys.data_ptr(), topk_w.data_ptr(), inv.data_ptr(), t, h, top_k, st)
    return out
