"""Engine ops: HIP/CDNA4 kernels for GPU tensors, PyTorch reference for CPU tensors.

Device dispatch only (no backend choice on the GPU): a CUDA tensor always goes to the
in-tree ``_C_kernels`` module and raises if it is not built -- there is no silent
eager fallback on the GPU.  Every GEMM of the forward path is hand-written too (ops/gemm.py:
gemm_wide / gemm_sq for decode-sized M, the persistent gemm_pf for prefill-sized M); torch's
F.linear remains only for shapes none of them takes (a bias, N not a multiple of 256).

Every wrapper checks dtype/contiguity/shape on the host before launching, and launches
on torch's current stream so the whole decode step can be captured in a HIP graph.
"""
from __future__ import annotations

from typing import Optional, Tuple


import torch

from .. import _ext, knobs
from . import gemm, quant
from . import reference as ref

__all__ = [
    "embedding", "rms_norm", "fused_add_rms_norm", "layer_norm", "linear", "silu_mul",
    "gelu_tanh", "rope_cache_append", "paged_attention_decode", "paged_attention_prefill",
    "argmax", "add_", "moe_route", "moe_mlp", "decode_split_plan", "paged_attention_decode_rope",
    "paged_attention_prefill_rope",
]


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _ck(t: torch.Tensor, name: str, dtype=torch.bfloat16):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


# --------------------------------------------------------------------- K1
def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    if not _gpu(weight):
        return ref.embedding(ids, weight)
    _ck(weight, "embedding.weight")
    _ck(ids, "embedding.ids", torch.int32)
    t, (v, h) = ids.numel(), weight.shape
    out = torch.empty(t, h, dtype=weight.dtype, device=weight.device)
    _ext.kernels().embedding(out.data_ptr(), ids.data_ptr(), weight.data_ptr(), t, h, v, _stream())
    return out


# --------------------------------------------------------------------- K2
def _q8_out(x_like: torch.Tensor):
    h = x_like.shape[-1]
    m = x_like.numel() // h
    return (torch.empty(m, h, dtype=quant.FP8, device=x_like.device),
            torch.empty(m, dtype=torch.float32, device=x_like.device))


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float, quant_out: bool = False):
    """``quant_out``: return the output as a per-token e4m3 :class:`quant.Fp8Act` for a W8A8 GEMM
    (quantized in the norm kernel's epilogue on the GPU)."""
    if not _gpu(x):
        y = ref.rms_norm(x, w, eps)
        return quant.Fp8Act(*quant.quantize_rows_ref(y), y.shape, y.dtype) if quant_out else y
    _ck(x, "rms_norm.x")
    _ck(w, "rms_norm.w")
    h = x.shape[-1]
    if quant_out:
        q, s = _q8_out(x)
        _ext.kernels().rms_norm_q8(0, x.data_ptr(), 0, w.data_ptr(), x.numel() // h, h, float(eps), q.data_ptr(),
                                   s.data_ptr(), _stream())
        return quant.Fp8Act(q, s, x.shape, x.dtype)
    y = torch.empty_like(x)
    _ext.kernels().rms_norm(y.data_ptr(), x.data_ptr(), 0, w.data_ptr(), x.numel() // h, h, float(eps), _stream())
    return y


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                       eps: float, quant_out: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """residual <- x + residual (in place); returns (rms_norm(residual) * w, residual).

    ``x`` may be a :class:`gemm.SplitKPartial` (split-K GEMM output not yet reduced): the
    reduction then happens inside the same kernel (splitk_add_rms_norm).  ``quant_out``: the
    normalised output comes back as a :class:`quant.Fp8Act` (see :func:`rms_norm`)."""
    if isinstance(x, gemm.SplitKPartial):
        _ck(residual, "fused_add_rms_norm.residual")
        _ck(w, "fused_add_rms_norm.w")
        if tuple(x.shape) != tuple(residual.shape):
            raise ValueError("x/residual shape mismatch")
        if quant_out:
            q, s = _q8_out(residual)
            _ext.kernels().splitk_add_rms_norm_q8(0, residual.data_ptr(), x.ws.data_ptr(), x.splits, x.m, x.n,
                                                  w.data_ptr(), float(eps), q.data_ptr(), s.data_ptr(), _stream())
            return quant.Fp8Act(q, s, residual.shape, residual.dtype), residual
        y = torch.empty_like(residual)
        _ext.kernels().splitk_add_rms_norm(y.data_ptr(), residual.data_ptr(), x.ws.data_ptr(), x.splits, x.m, x.n,
                                           w.data_ptr(), float(eps), _stream())
        return y, residual
    if not _gpu(x):
        y, residual = ref.fused_add_rms_norm(x, residual, w, eps)
        return (quant.Fp8Act(*quant.quantize_rows_ref(y), y.shape, y.dtype) if quant_out else y), residual
    _ck(x, "fused_add_rms_norm.x")
    _ck(residual, "fused_add_rms_norm.residual")
    _ck(w, "fused_add_rms_norm.w")
    if x.shape != residual.shape:
        raise ValueError("x/residual shape mismatch")
    h = x.shape[-1]
    if quant_out:
        q, s = _q8_out(x)
        _ext.kernels().rms_norm_q8(0, x.data_ptr(), residual.data_ptr(), w.data_ptr(), x.numel() // h, h,
                                   float(eps), q.data_ptr(), s.data_ptr(), _stream())
        return quant.Fp8Act(q, s, x.shape, x.dtype), residual
    y = torch.empty_like(x)
    _ext.kernels().rms_norm(y.data_ptr(), x.data_ptr(), residual.data_ptr(), w.data_ptr(), x.numel() // h, h,
                            float(eps), _stream())
    return y, residual


def layer_norm(x, w, b, eps):
    # GPT-2 plumbing config only: torch path on both devices.
    return ref.layer_norm(x, w, b, eps)


def gelu_tanh(x):
    return ref.gelu_tanh(x)


# --------------------------------------------------------------- GEMM
def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None, defer: bool = False):
    """y = x @ w^T (+bias). w is [N, K].  ``defer`` (GPU): the result may come back as a
    :class:`gemm.SplitKPartial` for ``fused_add_rms_norm`` to reduce (or ``materialize()``).
    ``w`` may be a :class:`quant.Fp8Weight` (W8A8 e4m3 GEMM, no bias)."""
    if isinstance(w, quant.Fp8Weight):
        if bias is not None:
            raise ValueError("linear: fp8 weights take no bias")
        return quant.linear_fp8(x, w, defer=defer)
    if not _gpu(x):
        return ref.linear(x, w, bias)
    return gemm.linear(x, w, bias, defer=defer)


def linear_swiglu(x: torch.Tensor, w_gate_up: torch.Tensor) -> torch.Tensor:
    """silu(x @ Wg^T) * (x @ Wu^T), W = [Wg; Wu]; fused into the GEMM epilogue on the GPU (decode)."""
    if isinstance(w_gate_up, quant.Fp8Weight):
        return quant.linear_fp8(x, w_gate_up, swiglu=True)
    if _gpu(x):
        from . import gemm
        y = gemm.linear_swiglu(x, w_gate_up)
        if y is not None:
            return y
    return silu_mul(linear(x, w_gate_up))


def add_(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """a <- a + b (in place)."""
    if not _gpu(a):
        a.copy_((a.float() + b.float()).to(a.dtype))
        return a
    _ck(a, "add_.a")
    _ck(b, "add_.b")
    if a.shape != b.shape:
        raise ValueError("add_: shape mismatch")
    _ext.kernels().add_inplace(a.data_ptr(), b.data_ptr(), a.numel(), _stream())
    return a


# ------------------------------------------------------------ SwiGLU
def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    if not _gpu(gu):
        return ref.silu_mul(gu)
    _ck(gu, "silu_mul.gu")
    t, two_i = gu.shape
    out = torch.empty(t, two_i // 2, dtype=gu.dtype, device=gu.device)
    _ext.kernels().silu_mul(out.data_ptr(), gu.data_ptr(), t, two_i // 2, _stream())
    return out


# ----------------------------------------------------------- K4 + K5
def rope_cache_append(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, num_heads, num_kv_heads,
                      head_dim, write_q: bool = True) -> Optional[torch.Tensor]:
    """Rotate k (and q) and append k / v^T to the paged cache; returns the rotated q [T, Hq, D], or
    None with ``write_q=False`` (the prefill attention then rotates q itself)."""
    if not _gpu(qkv):
        q = ref.rope_cache_append(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, num_heads,
                                  num_kv_heads, head_dim)
        return q if write_q else None
    _ck(qkv, "rope.qkv")
    _ck(k_cache, "k_cache")
    _ck(v_cache, "v_cache")
    _ck(positions, "positions", torch.int32)
    _ck(slot_mapping, "slot_mapping", torch.int32)
    t = qkv.shape[0]
    if qkv.shape[1] != (num_heads + 2 * num_kv_heads) * head_dim:
        raise ValueError("qkv width mismatch")
    if cos_sin is not None:
        _ck(cos_sin, "cos_sin", torch.float32)
        if cos_sin.shape[1] != head_dim:
            raise ValueError("cos_sin width must equal head_dim")
    q = torch.empty(t, num_heads, head_dim, dtype=qkv.dtype, device=qkv.device) if write_q else None
    _ext.kernels().rope_cache_append(q.data_ptr() if write_q else 0, qkv.data_ptr(), positions.data_ptr(),
                                     0 if cos_sin is None else cos_sin.data_ptr(), k_cache.data_ptr(),
                                     v_cache.data_ptr(), slot_mapping.data_ptr(), t, num_heads, num_kv_heads,
                                     head_dim, k_cache.shape[2], int(knobs.K.v_group_append), _stream())
    return q


# ---------------------------------------------------------- K6 / K7


def decode_split_plan(batch: int, num_kv_heads: int, max_ctx: int, block_size: int = 32,
                      max_blocks: Optional[int] = None, target_waves: Optional[int] = None) -> Tuple[int, int]:
    """(num_splits, split_len) for the decode kernel (one wave per split x kv-head x sequence).

    Aim for ~8 waves per CU (256 CUs) with >= 2 KV blocks per split so each wave's load
    pipeline has something to overlap.  The split BOUNDARIES depend only on the pow2-bucketed
    batch x kv-heads and on the block-table width -- not on ``max_ctx`` -- so a graph replayed
    at a padded (batch, context) bucket and the eager path partition every sequence's keys
    identically: the extra splits of the bucket are empty and add exact zeros, and the two
    paths produce bit-identical attention.
    """
    target_waves = target_waves or knobs.K.attn_target_waves     # sweep: profiles/attn_decode_sweep.txt
    max_blocks = max_blocks or -(-max_ctx // block_size)
    pairs = 1 << max(0, (max(1, batch * num_kv_heads) - 1).bit_length())
    target = max(1, min(64, target_waves // pairs))
    split_len = block_size * max(2, -(-max_blocks // target))
    splits = max(1, -(-max_ctx // split_len))
    return splits, split_len


def _into(out: Optional[torch.Tensor], y: torch.Tensor) -> torch.Tensor:
    if out is None:
        return y
    out.copy_(y)
    return out


def paged_attention_decode(q, k_cache, v_cache, block_tables, seq_lens, scale: float,
                           max_ctx: Optional[int] = None, workspace: Optional[tuple] = None,
                           out: Optional[torch.Tensor] = None):
    """``out``: write the result there (a contiguous [B, Hq, D] view, e.g. rows of a mixed step)."""
    if not _gpu(q):
        return _into(out, ref.paged_attention_decode(q, k_cache, v_cache, block_tables, seq_lens, scale))
    _ck(q, "attn.q")
    _ck(k_cache, "k_cache")
    _ck(v_cache, "v_cache")
    _ck(block_tables, "block_tables", torch.int32)
    _ck(seq_lens, "seq_lens", torch.int32)
    b, hq, d = q.shape
    hkv, bs = k_cache.shape[1], k_cache.shape[2]
    max_blocks = block_tables.shape[1]
    if max_ctx is None:
        max_ctx = max_blocks * bs
    if max_ctx > max_blocks * bs:
        raise ValueError("max_ctx exceeds block table capacity")
    splits, split_len = decode_split_plan(b, hkv, max_ctx, bs, max_blocks)
    if out is None:
        out = torch.empty_like(q)
    elif out.shape != q.shape or not out.is_contiguous() or out.dtype != q.dtype:
        raise ValueError("attention out must be a contiguous tensor shaped like q")
    po = pml = 0
    if splits > 1:
        if workspace is None:
            po_t = torch.empty(b * hq * splits * d, dtype=torch.float32, device=q.device)
            pml_t = torch.empty(b * hq * splits * 2, dtype=torch.float32, device=q.device)
        else:
            po_t, pml_t = workspace
            if po_t.numel() < b * hq * splits * d or pml_t.numel() < b * hq * splits * 2:
                raise ValueError("attention workspace too small")
        po, pml = po_t.data_ptr(), pml_t.data_ptr()
    _ext.kernels().paged_attention_decode(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                          block_tables.data_ptr(), seq_lens.data_ptr(), po, pml, b, hq, hkv, d,
                                          bs, max_blocks, splits, split_len, float(scale), _stream())
    return out


def paged_attention_decode_rope(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, block_tables, seq_lens,
                                num_heads: int, num_kv_heads: int, head_dim: int, scale: float,
                                max_ctx: Optional[int] = None, workspace: Optional[tuple] = None):
    """Decode attention with RoPE + KV-cache append fused in (one launch instead of two): reads the raw
    qkv projection [B, (Hq + 2 Hkv) * D], appends each sequence's new k / v at ``slot_mapping`` and
    attends over the whole context including it.  Same result as ``rope_cache_append`` followed by
    ``paged_attention_decode`` (the new key is folded in last instead of inside its block).

    ``qkv`` may be a :class:`gemm.SplitKPartial`: the kernel then sums the split-K slabs (f32 sums of f16 x 2^-6 slices) itself
    (bit-identical to reducing first), which removes the reduce launch and the bf16 round trip."""
    part = None
    if isinstance(qkv, gemm.SplitKPartial):
        part = qkv
        if len(part.shape) != 2:
            raise ValueError("qkv partial must be [B, (Hq + 2 Hkv) * D]")
        b, width, qdtype, qdev = part.m, part.n, part.dtype, part.device
    else:
        b, width, qdtype, qdev = qkv.shape[0], qkv.shape[-1], qkv.dtype, qkv.device
    if part is None and not _gpu(qkv):
        q = ref.rope_cache_append(qkv, positions, cos_sin, k_cache, v_cache, slot_mapping, num_heads, num_kv_heads,
                                  head_dim)
        return ref.paged_attention_decode(q, k_cache, v_cache, block_tables, seq_lens, scale)
    if part is None:
        _ck(qkv, "attn.qkv")
    _ck(k_cache, "k_cache")
    _ck(v_cache, "v_cache")
    _ck(positions, "positions", torch.int32)
    _ck(slot_mapping, "slot_mapping", torch.int32)
    _ck(block_tables, "block_tables", torch.int32)
    _ck(seq_lens, "seq_lens", torch.int32)
    hq, hkv, d = num_heads, num_kv_heads, head_dim
    if width != (hq + 2 * hkv) * d:
        raise ValueError("qkv width mismatch")
    if cos_sin is not None:
        _ck(cos_sin, "cos_sin", torch.float32)
        if cos_sin.shape[1] != d:
            raise ValueError("cos_sin width must equal head_dim")
    bs = k_cache.shape[2]
    max_blocks = block_tables.shape[1]
    if max_ctx is None:
        max_ctx = max_blocks * bs
    if max_ctx > max_blocks * bs:
        raise ValueError("max_ctx exceeds block table capacity")
    splits, split_len = decode_split_plan(b, hkv, max_ctx, bs, max_blocks)
    out = torch.empty(b, hq, d, dtype=qdtype, device=qdev)
    po = pml = 0
    if splits > 1:
        if workspace is None:
            po_t = torch.empty(b * hq * splits * d, dtype=torch.float32, device=qdev)
            pml_t = torch.empty(b * hq * splits * 2, dtype=torch.float32, device=qdev)
        else:
            po_t, pml_t = workspace
            if po_t.numel() < b * hq * splits * d or pml_t.numel() < b * hq * splits * 2:
                raise ValueError("attention workspace too small")
        po, pml = po_t.data_ptr(), pml_t.data_ptr()
    _ext.kernels().paged_attention_decode_rope(
        out.data_ptr(), 0 if part is not None else qkv.data_ptr(), positions.data_ptr(),
        0 if cos_sin is None else cos_sin.data_ptr(),
        slot_mapping.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(), seq_lens.data_ptr(),
        po, pml, b, hq, hkv, d, bs, max_blocks, splits, split_len, float(scale),
        0 if part is None else part.ws.data_ptr(), 0 if part is None else part.splits,
        0 if part is None else part.m * part.n, _stream())
    return out


def prefill_attn_version(max_q_len: int, head_dim: int) -> int:
    """The prefill attention kernel for a batch: knobs.prefill_attn, or with 0 (auto) from
    knobs.prefill_w32_min_q query rows at head_dim 128 the persistent 32x32x16 kernel (9: 1.1x v4 at
    64 x 512-token prompts, 1.35x at 1 x 16k; profiles/round6_attention.md) -- or its one-shot form (7)
    while spinning comm kernels hold CUs (ops.gemm.reserve_cus_for_comm: a persistent grid sized to
    every CU would wait for them) -- and v4 below (256 x 128-token prompts: v4 180-185 us, v9 185-193)."""
    v = knobs.K.prefill_attn
    if v:
        return v
    if head_dim != 128 or max_q_len < knobs.K.prefill_w32_min_q:
        return 4
    from . import gemm
    return 7 if gemm._comm_cus else 9


def paged_attention_prefill(q, k_cache, v_cache, block_tables, cu_seqlens_q, seq_lens, scale: float,
                            max_q_len: Optional[int] = None, version: int = 0, out: Optional[torch.Tensor] = None):
    """``version``: prefill kernel 3, 4, 6, 7 or 9 (0: prefill_attn_version); ``out`` as paged_attention_decode."""
    if not _gpu(q):
        return _into(out, ref.paged_attention_prefill(q, k_cache, v_cache, block_tables, cu_seqlens_q, seq_lens,
                                                      scale))
    _ck(q, "attn.q")
    _ck(k_cache, "k_cache")
    _ck(v_cache, "v_cache")
    _ck(block_tables, "block_tables", torch.int32)
    _ck(cu_seqlens_q, "cu_seqlens_q", torch.int32)
    _ck(seq_lens, "seq_lens", torch.int32)
    t, hq, d = q.shape
    b = seq_lens.shape[0]
    if max_q_len is None:
        max_q_len = int((cu_seqlens_q[1:] - cu_seqlens_q[:-1]).max().item()) if b else 0
    if out is None:
        out = torch.empty_like(q)
    elif out.shape != q.shape or not out.is_contiguous() or out.dtype != q.dtype:
        raise ValueError("attention out must be a contiguous tensor shaped like q")
    _ext.kernels().paged_attention_prefill(out.data_ptr(), q.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                           block_tables.data_ptr(), cu_seqlens_q.data_ptr(), seq_lens.data_ptr(),
                                           b, hq, k_cache.shape[1], d, k_cache.shape[2], block_tables.shape[1],
                                           int(max_q_len), float(scale), version or prefill_attn_version(int(max_q_len), d),
                                           0, 0, 0,
                                           _stream())
    return out


PF_MAX_CHUNKS = 1024    # attention.hip kPfMaxChunks: the LDS prefill kernel stages <= 32k tokens of block ids


def prefill_rope_in_attention(max_blocks: Optional[int] = None) -> bool:
    """Prefill q-RoPE inside the attention kernel (knobs.prefill_fused_rope; LDS kernel versions).
    ``max_blocks``: the batch's block-table width -- beyond ``PF_MAX_CHUNKS`` (32k-token sequences)
    the launcher falls back to the register-tiled kernel, which reads a rotated q, so the caller
    must take ``rope_cache_append(write_q=True)`` + the plain prefill kernel instead."""
    if max_blocks is not None and max_blocks > PF_MAX_CHUNKS:
        return False
    return knobs.K.prefill_fused_rope and knobs.K.prefill_attn in (0, 4, 6, 7, 9)


def paged_attention_prefill_rope(qkv, positions, cos_sin, k_cache, v_cache, block_tables, cu_seqlens_q, seq_lens,
                                 num_heads: int, head_dim: int, scale: float, max_q_len: Optional[int] = None,
                                 out: Optional[torch.Tensor] = None):
    """Prefill attention reading q straight from the qkv projection [T, (Hq + 2 Hkv) * D] and rotating it
    in registers (K / V already appended by ``rope_cache_append(..., write_q=False)``): the rotated q
    never round-trips through HBM.  Returns [T, Hq, D]."""
    hkv = k_cache.shape[1]
    t, width = qkv.shape
    if not _gpu(qkv):
        q = ref.rope_q(qkv, positions, cos_sin, num_heads, head_dim)
        return _into(out, ref.paged_attention_prefill(q, k_cache, v_cache, block_tables, cu_seqlens_q, seq_lens,
                                                      scale))
    _ck(qkv, "attn.qkv")
    _ck(k_cache, "k_cache")
    _ck(v_cache, "v_cache")
    _ck(block_tables, "block_tables", torch.int32)
    _ck(cu_seqlens_q, "cu_seqlens_q", torch.int32)
    _ck(seq_lens, "seq_lens", torch.int32)
    _ck(positions, "positions", torch.int32)
    if width != (num_heads + 2 * hkv) * head_dim:
        raise ValueError("qkv width mismatch")
    if cos_sin is not None:
        _ck(cos_sin, "cos_sin", torch.float32)
    if not prefill_rope_in_attention(block_tables.shape[1]):
        raise ValueError("in-kernel prefill RoPE needs an LDS prefill kernel (knobs.prefill_attn 0, 4, 6, 7 or 9) and "
                         f"block tables of <= {PF_MAX_CHUNKS} blocks")
    b = seq_lens.shape[0]
    if max_q_len is None:
        max_q_len = int((cu_seqlens_q[1:] - cu_seqlens_q[:-1]).max().item()) if b else 0
    if out is None:
        out = torch.empty(t, num_heads, head_dim, dtype=qkv.dtype, device=qkv.device)
    _ext.kernels().paged_attention_prefill(out.data_ptr(), qkv.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                           block_tables.data_ptr(), cu_seqlens_q.data_ptr(), seq_lens.data_ptr(),
                                           b, num_heads, hkv, head_dim, k_cache.shape[2], block_tables.shape[1],
                                           int(max_q_len), float(scale), prefill_attn_version(int(max_q_len), head_dim),
                                           positions.data_ptr(),
                                           0 if cos_sin is None else cos_sin.data_ptr(), width, _stream())
    return out


# ------------------------------------------------------------- K10
def argmax(logits: torch.Tensor) -> torch.Tensor:
    if not _gpu(logits):
        return ref.argmax(logits)
    if logits.dtype != torch.bfloat16:
        return logits.argmax(-1).to(torch.int32)
    if logits.stride(-1) != 1:
        raise ValueError("argmax: last dim must be contiguous")
    rows, v = logits.shape
    out = torch.empty(rows, dtype=torch.int32, device=logits.device)
    _ext.kernels().argmax(out.data_ptr(), logits.data_ptr(), rows, v, logits.stride(0), _stream())
    return out


# ------------------------------------------------------------ K11/K12
def moe_route(router_logits: torch.Tensor, top_k: int):
    from . import moe
    return moe.route(router_logits, top_k)


def moe_mlp(x, w_gate_up, w_down, topk_w, topk_ids):
    from . import moe
    return moe.mlp(x, w_gate_up, w_down, topk_w, topk_ids)


def moe_forward(x, w_router, w_gate_up, w_down, top_k: int, expert_offset: int = 0):
    """Full Mixtral sparse MLP: route + expert SwiGLU MLPs + weighted combine (``expert_offset``:
    the weights hold experts [offset, offset + E_local) -- expert parallelism, ops/moe.py)."""
    from . import moe
    return moe.forward(x, w_router, w_gate_up, w_down, top_k, expert_offset)
