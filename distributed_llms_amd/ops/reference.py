"""Plain-PyTorch implementations of every engine op.

Two roles:
  * the CPU execution path (CPU workers, the GPT-2 plumbing config, CPU tests);
  * the numerics oracle the HIP kernels are tested against (run in fp32).

They replace what the reference delegates to ``torch.matmul`` inside its
placeholder ``ModelShard.compute`` (``src/worker/node.py:24-32``) with the real
transformer-block math.

Paged-KV layout (shared with the HIP kernels, one tensor pair per layer):
  k_cache: [num_blocks, num_kv_heads, block_size, head_dim]
  v_cache: [num_blocks, num_kv_heads, head_dim, block_size]   (32-key blocks: K row / V^T element
                                                              order of csrc/kernels/common.h krow32 /
                                                              vofs, a [4][D][8] V^T tile; V stored transposed
           so the P·V MFMA reads token-contiguous 16-byte fragments)
``slot = block_id * block_size + offset`` addresses one token's K/V.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F


def embedding(ids: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    return weight.index_select(0, ids.long())


def rms_norm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype)


def fused_add_rms_norm(x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                       eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """residual <- x + residual ; returns (rms_norm(residual) * w, residual)."""
    r = (x.float() + residual.float())
    residual.copy_(r.to(residual.dtype))
    r = residual.float()
    y = r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + eps)
    return (y * w.float()).to(x.dtype), residual


def layer_norm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = x @ w^T (+ bias); w is [out, in] (nn.Linear convention)."""
    if x.device.type == "cpu" and x.dtype in (torch.bfloat16, torch.float16):
        y = x.float() @ w.float().t()
        if bias is not None:
            y = y + bias.float()
        return y.to(x.dtype)
    return F.linear(x, w, bias)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    """gu = [gate | up] along the last dim -> silu(gate) * up."""
    i = gu.shape[-1] // 2
    g, u = gu[..., :i].float(), gu[..., i:].float()
    return (F.silu(g) * u).to(gu.dtype)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def rope_cos_sin(head_dim: int, max_pos: int, theta: float, scaling: Optional[dict] = None,
                 device="cpu") -> torch.Tensor:
    """[max_pos, head_dim] float32: first half cos, second half sin (rotate-half RoPE).

    Implements the ``llama3`` frequency rescaling when ``scaling['rope_type'] == 'llama3'``.
    """
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.float64) / head_dim))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        lo, hi = scaling["low_freq_factor"], scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    freqs = torch.outer(t, inv)
    return torch.cat([freqs.cos(), freqs.sin()], dim=-1).float().to(device)


def apply_rope(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, D]; rotate-half convention (HF Llama)."""
    d = x.shape[-1]
    cs = cos_sin.index_select(0, pos.long())          # [T, D]
    cos, sin = cs[:, : d // 2].unsqueeze(1), cs[:, d // 2:].unsqueeze(1)
    xf = x.float()
    x1, x2 = xf[..., : d // 2], xf[..., d // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def rope_q(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: Optional[torch.Tensor], num_heads: int,
           head_dim: int) -> torch.Tensor:
    """The rotated q [T, Hq, D] of a fused qkv projection."""
    t = qkv.shape[0]
    q = qkv[:, : num_heads * head_dim].view(t, num_heads, head_dim)
    return apply_rope(q, positions, cos_sin) if cos_sin is not None else q.contiguous()


def rope_cache_append(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: Optional[torch.Tensor],
                      k_cache: torch.Tensor, v_cache: torch.Tensor, slot_mapping: torch.Tensor,
                      num_heads: int, num_kv_heads: int, head_dim: int) -> torch.Tensor:
    """Split fused qkv [T, (Hq+2Hkv)D], rotate q/k, scatter k/v into the paged cache, return q."""
    t = qkv.shape[0]
    q = qkv[:, : num_heads * head_dim].view(t, num_heads, head_dim)
    k = qkv[:, num_heads * head_dim: (num_heads + num_kv_heads) * head_dim].view(t, num_kv_heads, head_dim)
    v = qkv[:, (num_heads + num_kv_heads) * head_dim:].view(t, num_kv_heads, head_dim)
    if cos_sin is not None:
        q = apply_rope(q, positions, cos_sin)
        k = apply_rope(k, positions, cos_sin)
    else:
        q = q.contiguous()
    bs = k_cache.shape[2]
    slots = slot_mapping.long()
    blk, off = slots // bs, slots % bs
    if bs == 32:
        k_cache[blk, :, _KROW32.to(off.device)[off], :] = k.to(k_cache.dtype)
        nb, hkv, d = v_cache.shape[0], v_cache.shape[1], v_cache.shape[2]
        v_cache.view(nb, hkv, 4, d, 8)[blk, :, off // 8, :, off % 8] = v.to(v_cache.dtype)
    else:
        k_cache[blk, :, off, :] = k.to(k_cache.dtype)
        v_cache[blk, :, :, off] = v.to(v_cache.dtype)
    return q


def _krow32() -> torch.Tensor:
    """Physical row of key j in a 32-key K block (csrc/kernels/common.h krow32)."""
    j = torch.arange(32)
    return ((j & 4) << 2) + ((j >> 3) << 2) + (j & 3)


_KROW32 = _krow32()


def _gather_kv(k_cache, v_cache, block_table, n):
    bs = k_cache.shape[2]
    nb = (n + bs - 1) // bs
    blocks = block_table[:nb].long()
    kb, vb = k_cache[blocks], v_cache[blocks]
    hkv, d = k_cache.shape[1], k_cache.shape[3]
    if bs == 32:
        kb = kb[:, :, _KROW32.to(kb.device), :]          # physical rows back to key order
        v = vb.reshape(nb, hkv, 4, d, 8).permute(1, 0, 2, 4, 3).reshape(hkv, nb * bs, d)[:, :n]
    else:
        v = vb.permute(1, 0, 3, 2).reshape(hkv, nb * bs, -1)[:, :n]
    k = kb.permute(1, 0, 2, 3).reshape(hkv, nb * bs, -1)[:, :n]
    return k, v  # [Hkv, n, D]


def paged_attention_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                           block_tables: torch.Tensor, seq_lens: torch.Tensor,
                           scale: float) -> torch.Tensor:
    """q [B, Hq, D] (one new token per sequence, already in the cache) -> [B, Hq, D].

    The whole batch in one gather: every sequence's first ceil(max_len / bs) blocks (table
    padding is block 0, a valid index), keys past its own length masked to -inf.
    """
    b, hq, d = q.shape
    if b == 0:
        return torch.empty_like(q)
    hkv, bs = k_cache.shape[1], k_cache.shape[2]
    lens = seq_lens[:b].long()
    n = int(lens.max())
    nb = (n + bs - 1) // bs
    blocks = block_tables[:b, :nb].long().clamp_min(0)
    kb, vb = k_cache[blocks], v_cache[blocks]               # [B, nb, Hkv, ...]
    if bs == 32:
        kb = kb[:, :, :, _KROW32.to(kb.device), :]         # physical rows back to key order
        v = vb.reshape(b, nb, hkv, 4, d, 8).permute(0, 2, 1, 3, 5, 4).reshape(b, hkv, nb * bs, d)
    else:
        v = vb.permute(0, 2, 1, 4, 3).reshape(b, hkv, nb * bs, d)
    k = kb.permute(0, 2, 1, 3, 4).reshape(b, hkv, nb * bs, d)
    qf = q.float().view(b, hkv, hq // hkv, d)
    s = torch.einsum("bhgd,bhnd->bhgn", qf, k.float()) * scale
    pad = torch.arange(nb * bs, device=q.device).view(1, 1, 1, -1) >= lens.to(q.device).view(b, 1, 1, 1)
    p = torch.softmax(s.masked_fill(pad, float("-inf")), dim=-1)
    o = torch.einsum("bhgn,bhnd->bhgd", p, v.float())
    return o.reshape(b, hq, d).to(q.dtype)


def paged_attention_prefill(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor,
                            block_tables: torch.Tensor, cu_seqlens_q: torch.Tensor,
                            seq_lens: torch.Tensor, scale: float) -> torch.Tensor:
    """Causal varlen attention for a packed chunk of prompts.

    q [T, Hq, D]; sequence i owns q rows cu_seqlens_q[i]:cu_seqlens_q[i+1], which are its
    LAST q_len tokens out of seq_lens[i] context tokens (all already in the cache).
    """
    t, hq, d = q.shape
    hkv = k_cache.shape[1]
    out = torch.empty_like(q)
    cu = cu_seqlens_q.tolist()
    for i in range(len(cu) - 1):
        s0, s1 = cu[i], cu[i + 1]
        ql = s1 - s0
        if ql == 0:
            continue
        n = int(seq_lens[i])
        k, v = _gather_kv(k_cache, v_cache, block_tables[i], n)
        qi = q[s0:s1].float().permute(1, 0, 2).reshape(hkv, hq // hkv, ql, d)
        s = torch.einsum("hgqd,hnd->hgqn", qi, k.float()) * scale
        qpos = torch.arange(n - ql, n, device=q.device).view(ql, 1)
        kpos = torch.arange(n, device=q.device).view(1, n)
        s = s.masked_fill(kpos > qpos, float("-inf"))
        p = torch.softmax(s, dim=-1)
        o = torch.einsum("hgqn,hnd->hgqd", p, v.float())
        out[s0:s1] = o.reshape(hq, ql, d).permute(1, 0, 2).to(q.dtype)
    return out


def argmax(logits: torch.Tensor) -> torch.Tensor:
    return logits.float().argmax(dim=-1).to(torch.int32)


def moe_route(router_logits: torch.Tensor, top_k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Mixtral routing: softmax over experts, top-k, renormalise. -> (weights f32, ids i32)."""
    probs = torch.softmax(router_logits.float(), dim=-1)
    w, ids = torch.topk(probs, top_k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def moe_mlp(x: torch.Tensor, w_gate_up: torch.Tensor, w_down: torch.Tensor,
            topk_w: torch.Tensor, topk_ids: torch.Tensor) -> torch.Tensor:
    """x [T,H]; w_gate_up [E, 2I, H]; w_down [E, H, I] -> [T, H] (weighted sum over top-k)."""
    t, h = x.shape
    out = torch.zeros(t, h, dtype=torch.float32, device=x.device)
    for e in range(w_gate_up.shape[0]):
        tok, slot = (topk_ids == e).nonzero(as_tuple=True)
        if tok.numel() == 0:
            continue
        gu = linear(x[tok], w_gate_up[e])
        y = linear(silu_mul(gu), w_down[e])
        out.index_add_(0, tok, y.float() * topk_w[tok, slot].unsqueeze(1).float())
    return out.to(x.dtype)
