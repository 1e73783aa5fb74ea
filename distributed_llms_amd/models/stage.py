"""A pipeline stage of a decoder-only transformer: the layer slice one worker owns.

Realizes what the reference's ``ModelShard`` only pretends to do
(``src/worker/node.py:13-32``: a placeholder ``inputs[key] @ param``): a contiguous
block range ``[layer_start, layer_end)`` with its paged KV cache, plus the token
embedding on the first stage and final norm + LM head on the last.

Stage I/O:
  first stage  input: token ids [T] int32
  other stages input: hidden [T, H] (the closed residual stream of the previous stage), or
                      [T, H + W] when the cut falls inside a half (sub-layer units): the residual
                      stream and the pending W-wide qkv / attention output / partial MLP sum
  last stage  output: logits [n, V] for the rows in ``meta.logits_idx``
  other stages output: hidden [T, H] or [T, H + W], as above
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from .. import knobs, ops
from ..config import ModelConfig
from ..ops import reference as ref
from . import weights as W

# knobs.fused_rope: decode RoPE + KV append fused into the attention kernel (one launch).  Split-K
# partials handed to the consumer instead of reduced by a separate launch: knobs.defer_qkv (the
# fused decode attention kernel sums them: every wave re-reads S slabs on its critical path, -3 %
# at B=256, off), knobs.defer_o (the MLP half's add + RMSNorm, +1 %).


@dataclass
class BatchMeta:
    """Per-step attention metadata (device tensors) + host-side scalars."""
    is_prefill: bool
    positions: torch.Tensor          # [T] int32
    slot_mapping: torch.Tensor       # [T] int32
    block_tables: torch.Tensor       # [B, max_blocks] int32
    seq_lens: torch.Tensor           # [B] int32 context length after this step
    cu_seqlens_q: Optional[torch.Tensor] = None   # [B+1] int32 (prefill)
    logits_idx: Optional[torch.Tensor] = None     # [B] int64 rows that produce logits (prefill)
    max_q_len: int = 1
    max_ctx: int = 0
    num_seqs: int = 0
    num_tokens: int = 0
    attn_workspace: Optional[tuple] = None
    # mixed prefill + decode step (is_prefill True): sequences [0, num_decode) are one-token decode
    # rows; cu_seqlens_p / max_q_len_p describe the prefill rows after them, max_ctx_d the decode
    # rows' longest context
    num_decode: int = 0
    cu_seqlens_p: Optional[torch.Tensor] = None
    max_ctx_d: int = 0
    max_q_len_p: int = 0


class KVCache:
    """Paged KV for the stage's layers: k [L, NB, Hkv, BS, D], v [L, NB, Hkv, D, BS]."""

    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int,
                 block_size: int, dtype, device):
        self.num_layers, self.num_blocks, self.block_size = num_layers, num_blocks, block_size
        self.k = torch.zeros(num_layers, num_blocks, num_kv_heads, block_size, head_dim, dtype=dtype, device=device)
        self.v = torch.zeros(num_layers, num_blocks, num_kv_heads, head_dim, block_size, dtype=dtype, device=device)

    def layer(self, i: int):
        return self.k[i], self.v[i]

    @property
    def nbytes(self) -> int:
        return self.k.numel() * self.k.element_size() * 2

    @staticmethod
    def bytes_per_block(num_layers, num_kv_heads, head_dim, block_size, dtype_bytes=2) -> int:
        return 2 * num_layers * num_kv_heads * head_dim * block_size * dtype_bytes


# A layer is five ATOMS: 0 norm + qkv projection, 1 RoPE + KV append + attention, 2 o-projection,
# 3 / 4 the MLP over the first / second half of the intermediate columns.  A stage's unit range is
# counted in units of ``unit_group`` per layer: 2 (halves: unit 0 = atoms 0-2, unit 1 = atoms 3-4)
# or 5 (one unit per atom; parallel/planner.py).
QKV_KEYS = {"attn_norm", "wqkv", "ln1_w", "ln1_b", "bqkv"}
O_KEYS = {"wo", "bo"}
ATTN_KEYS = QKV_KEYS | O_KEYS
NATOM = 5
_HALF_ATOM = (0, 3)          # first atom of half-unit j


def unit_to_atom(u: int, group: int) -> int:
    if group == NATOM:
        return u
    if group != 2:
        raise ValueError(f"unit group must be 2 or {NATOM}")
    return NATOM * (u // 2) + _HALF_ATOM[u % 2]


class ModelStage:
    """Layers ``[layer_start, layer_end)``, or -- finer -- half-layer *units* ``[u0, u1)``:
    unit 2l is the attention half of layer l (norm, qkv, RoPE + KV append, attention, o-proj),
    unit 2l+1 its MLP half (``unit_group`` 2), or sub-layer atoms (``unit_group`` 5, see NATOM).
    Pipeline stages may start or end in the middle of a layer; at a half boundary the hand-off is
    the closed residual stream ([T, H]), at a cut inside a half it is [T, H + W] (``in_width`` /
    ``out_width``)."""

    def __init__(self, cfg: ModelConfig, layer_start: int, layer_end: int, device="cpu",
                 dtype=torch.bfloat16, units: Optional[tuple] = None, tp=None, unit_group: int = 2):
        """``tp``: a :class:`~distributed_llms_amd.parallel.tensor_parallel.TPGroup` -- this rank then
        holds its column / row / vocab shard of every layer (parallel/tensor_parallel.py).
        ``units``: [u0, u1) in units of ``unit_group`` per layer (2 halves or 5 sub-layer atoms)."""
        from ..parallel.tensor_parallel import TPGroup, check_divisible
        self.tp = tp if tp is not None else TPGroup(0, 1)
        check_divisible(cfg, self.tp.size, self.tp.moe)
        # heads this rank computes (all of them without TP)
        self.hq = cfg.num_heads // self.tp.size
        self.hkv = cfg.num_kv_heads // self.tp.size
        self.q_size_local = self.hq * cfg.head_dim
        g = int(unit_group)
        if units is None:
            units = (g * layer_start, g * layer_end)
        u0, u1 = int(units[0]), int(units[1])
        if not (0 <= u0 < u1 <= g * cfg.num_layers):
            raise ValueError(f"bad unit range [{u0}, {u1}) for {cfg.num_layers} layers")
        self.cfg = cfg
        self.unit_group = g
        self.unit_start, self.unit_end = u0, u1
        # the same range in atoms (5 per layer)
        self.atom_start, self.atom_end = unit_to_atom(u0, g), unit_to_atom(u1, g)
        a0, a1 = self.atom_start, self.atom_end
        if a0 % NATOM not in (0, 3) or a1 % NATOM not in (0, 3):
            if cfg.arch == "gpt2" or cfg.is_moe:
                raise ValueError("sub-layer cuts need a dense SwiGLU model")
            if self.tp.enabled:
                raise ValueError("sub-layer cuts are not combined with tensor parallelism")
        self.layer_start, self.layer_end = a0 // NATOM, (a1 + NATOM - 1) // NATOM
        self.is_first = a0 == 0
        self.is_last = a1 == NATOM * cfg.num_layers
        # layers whose attention core (and therefore KV cache) lives on this stage
        self.kv_layers = [l for l in range(self.layer_start, self.layer_end) if self.has(l, 1)]
        self.kv_index = {l: i for i, l in enumerate(self.kv_layers)}
        self.device = torch.device(device)
        self.dtype = dtype
        self.layers: List[Dict[str, torch.Tensor]] = []
        self.embed: Dict[str, torch.Tensor] = {}
        self.head: Dict[str, torch.Tensor] = {}
        self.kv: Optional[KVCache] = None
        self.cos_sin = None
        if cfg.arch != "gpt2":
            self.cos_sin = ref.rope_cos_sin(cfg.head_dim, cfg.max_position, cfg.rope_theta, cfg.rope_scaling,
                                            device=self.device)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)

    # --------------------------------------------------------------- weights
    @property
    def num_layers(self) -> int:
        """Layers with KV on this stage (what the paged KV pool is sized for)."""
        return len(self.kv_layers)

    def has(self, layer: int, atom: int) -> bool:
        """Does this stage run atom ``atom`` (0..4, see NATOM) of ``layer``?"""
        return self.atom_start <= NATOM * layer + atom < self.atom_end

    def _keep(self, layer: int, name: str) -> bool:
        if name in QKV_KEYS:
            return self.has(layer, 0)
        if name in O_KEYS:
            return self.has(layer, 2)
        return self.has(layer, 3) or self.has(layer, 4)

    def aux_width(self, atom: int) -> int:
        """Width of the pending tensor a cut before global atom ``atom`` hands over (0: none)."""
        j = atom % NATOM
        if j == 1:
            return (self.hq + 2 * self.hkv) * self.cfg.head_dim     # qkv projection output
        if j == 2:
            return self.q_size_local                                  # attention output
        if j == 4:
            return self.cfg.hidden_size                               # partial MLP sum
        return 0

    @property
    def in_width(self) -> int:
        """Columns of this stage's hidden input (non-first stages)."""
        return self.cfg.hidden_size + self.aux_width(self.atom_start)

    @property
    def out_width(self) -> int:
        return self.cfg.hidden_size + (0 if self.is_last else self.aux_width(self.atom_end))

    def _slice_mlp_halves(self):
        """A stage holding one MLP half of a layer keeps only that half's intermediate columns:
        rows [c0, c1) of the gate and of the up block of w_gate_up, columns [c0, c1) of w_down."""
        i = self.cfg.intermediate_size
        for l, lw in zip(range(self.layer_start, self.layer_end), self.layers):
            h0, h1 = self.has(l, 3), self.has(l, 4)
            if h0 == h1 or "w_gate_up" not in lw:
                continue
            c0, c1 = (0, i // 2) if h0 else (i // 2, i)
            gu = lw["w_gate_up"]
            lw["w_gate_up"] = torch.cat([gu[c0:c1], gu[i + c0:i + c1]], 0).contiguous()
            lw["w_down"] = lw["w_down"][:, c0:c1].contiguous()

    def needs_embed(self) -> bool:
        return self.is_first or (self.is_last and self.cfg.tie_embeddings)

    def _shard(self):
        """Keep this tensor-parallel rank's shard of every layer and of the LM head (the full
        tensors are generated / loaded first, so shards are slices of the same model)."""
        if not self.tp.enabled:
            return
        from ..parallel.tensor_parallel import shard_block, shard_vocab
        r, n = self.tp.rank, self.tp.size
        self.layers = [shard_block(self.cfg, lw, r, n, self.tp.moe) for lw in self.layers]
        if self.is_last:
            self.head["lm_head_tp"] = shard_vocab(self.lm_head_weight(full=True), r, n)
            self.head.pop("lm_head", None)

    def init_synthetic(self, seed: int = 0) -> "ModelStage":
        """Seeded random-init weights generated directly on the stage's device."""
        cfg = self.cfg
        self.layers = []
        for l in range(self.layer_start, self.layer_end):
            shapes = {n: s for n, s in W.block_shapes(cfg).items() if self._keep(l, n)}
            lw = {n: W.synth_tensor(seed, l, n, s, self.dtype, self.device) for n, s in shapes.items()}
            if self.tp.enabled:
                from ..parallel.tensor_parallel import shard_block
                lw = shard_block(cfg, lw, self.tp.rank, self.tp.size, self.tp.moe)   # one full layer at a time
            self.layers.append(lw)
        self._slice_mlp_halves()
        if self.needs_embed():
            self.embed = W.synth_embed(cfg, seed, self.dtype, self.device)
            if not self.is_first:
                self.embed.pop("pos_embed", None)
        if self.is_last:
            self.head = W.synth_head(cfg, seed, self.dtype, self.device)
            if self.tp.enabled:
                from ..parallel.tensor_parallel import shard_vocab
                self.head["lm_head_tp"] = shard_vocab(self.lm_head_weight(full=True), self.tp.rank, self.tp.size)
                self.head.pop("lm_head", None)
        return self

    def load_hf_state(self, sd: Dict[str, torch.Tensor]) -> "ModelStage":
        """Load from HF-named tensors (a shard file's dict); fuses q|k|v and gate|up."""
        cfg = self.cfg
        conv = lambda t: t.to(device=self.device, dtype=self.dtype).contiguous()
        self.layers = [{k: conv(v) for k, v in W.hf_to_block(cfg, l, sd).items() if self._keep(l, k)}
                       for l in range(self.layer_start, self.layer_end)]
        self._slice_mlp_halves()
        if self.needs_embed():
            names = W.hf_embed_names(cfg)
            if not self.is_first:           # tied LM head on the last stage: token table only
                names = {"embed": names["embed"]}
            self.embed = {k: conv(sd[n]) for k, n in names.items()}
        if self.is_last:
            self.head = {k: conv(sd[n]) for k, n in W.hf_head_names(cfg).items()}
        self._shard()
        return self

    def quantize(self, mode: str) -> "ModelStage":
        """``"fp8"``: the dense projections (qkv, o, gate|up, down) and MoE expert stacks become
        W8A8 e4m3 weights (ops/quant.py); embeddings, norms, router, LM head and the KV cache stay
        in ``dtype``."""
        if mode in ("", "none", None):
            return self
        if mode != "fp8":
            raise ValueError(f"unknown quantization {mode!r} (none, fp8)")
        from ..ops import quant
        quant.quantize_layers(self.layers)
        return self

    @staticmethod
    def _nbytes(t) -> int:
        return t.nbytes() if hasattr(t, "scale") else t.numel() * t.element_size()

    def weight_bytes(self) -> int:
        n = sum(self._nbytes(t) for d in self.layers for t in d.values())
        n += sum(t.numel() * t.element_size() for t in self.embed.values())
        n += sum(t.numel() * t.element_size() for t in self.head.values())
        return n

    def allocate_kv(self, num_blocks: int, block_size: int) -> KVCache:
        cfg = self.cfg
        self.kv = KVCache(self.num_layers, num_blocks, self.hkv, cfg.head_dim, block_size,
                          self.dtype, self.device)
        return self.kv

    def lm_head_weight(self, full: bool = False) -> torch.Tensor:
        """The LM head rows this rank computes (its vocab shard under TP; ``full``: all rows)."""
        if not full and "lm_head_tp" in self.head:
            return self.head["lm_head_tp"]
        return self.embed["embed"] if self.cfg.tie_embeddings else self.head["lm_head"]

    # --------------------------------------------------------------- forward
    @torch.inference_mode()
    def forward(self, inp: torch.Tensor, meta: BatchMeta) -> torch.Tensor:
        if self.kv is None:
            raise RuntimeError("allocate_kv() before forward()")
        if self.cfg.arch == "gpt2":
            return self._forward_gpt2(inp, meta)
        return self._forward_llama(inp, meta)

    def _attention(self, qkv, li: int, meta: BatchMeta) -> torch.Tensor:
        """``qkv``: [T, (Hq + 2 Hkv) D] or, from a split-K projection, a SplitKPartial that the fused
        decode kernel reduces itself (any other path materialises it)."""
        cfg = self.cfg
        k_cache, v_cache = self.kv.layer(li)
        fused = not meta.is_prefill and knobs.K.fused_rope and \
            (isinstance(qkv, ops.gemm.SplitKPartial) or qkv.is_cuda)
        if not fused and isinstance(qkv, ops.gemm.SplitKPartial):
            qkv = qkv.materialize()
        if fused:
            o = ops.paged_attention_decode_rope(qkv, meta.positions, self.cos_sin, k_cache, v_cache, meta.slot_mapping,
                                                meta.block_tables, meta.seq_lens, self.hq, self.hkv,
                                                cfg.head_dim, self.scale, max_ctx=meta.max_ctx or None,
                                                workspace=meta.attn_workspace)
            return o.view(o.shape[0], self.q_size_local)
        if meta.is_prefill and not meta.num_decode and qkv.is_cuda and \
                ops.prefill_rope_in_attention(meta.block_tables.shape[1]):
            ops.rope_cache_append(qkv, meta.positions, self.cos_sin, k_cache, v_cache, meta.slot_mapping,
                                  self.hq, self.hkv, cfg.head_dim, write_q=False)
            o = ops.paged_attention_prefill_rope(qkv, meta.positions, self.cos_sin, k_cache, v_cache,
                                                 meta.block_tables, meta.cu_seqlens_q, meta.seq_lens, self.hq,
                                                 cfg.head_dim, self.scale, max_q_len=meta.max_q_len)
            return o.view(o.shape[0], self.q_size_local)
        q = ops.rope_cache_append(qkv, meta.positions, self.cos_sin, k_cache, v_cache, meta.slot_mapping,
                                  self.hq, self.hkv, cfg.head_dim)
        if meta.is_prefill and meta.num_decode:
            # mixed step: decode rows through the split-KV decode kernel, prefill chunks through
            # the prefill kernel (both read the cache the append above just completed)
            nd = meta.num_decode
            o = torch.empty_like(q)
            ops.paged_attention_decode(q[:nd], k_cache, v_cache, meta.block_tables[:nd], meta.seq_lens[:nd],
                                       self.scale, max_ctx=meta.max_ctx_d or None, out=o[:nd])
            ops.paged_attention_prefill(q[nd:], k_cache, v_cache, meta.block_tables[nd:], meta.cu_seqlens_p,
                                        meta.seq_lens[nd:], self.scale, max_q_len=meta.max_q_len_p, out=o[nd:])
            return o.view(o.shape[0], self.q_size_local)
        if meta.is_prefill:
            o = ops.paged_attention_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_seqlens_q,
                                            meta.seq_lens, self.scale, max_q_len=meta.max_q_len)
        else:
            o = ops.paged_attention_decode(q, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.scale,
                                           max_ctx=meta.max_ctx or None, workspace=meta.attn_workspace)
        return o.view(o.shape[0], self.q_size_local)

    def _mlp(self, h: torch.Tensor, lw: Dict[str, torch.Tensor]) -> torch.Tensor:
        if self.cfg.is_moe:
            out = ops.moe_forward(h, lw["router"], lw["experts_gate_up"], lw["experts_down"],
                                  self.cfg.experts_per_token, self.tp.expert_offset(self.cfg.num_experts))
            return self.tp.all_reduce_(out) if self.tp.enabled else out
        # defer: the down projection's split-K reduce is fused into the next residual-add + RMSNorm
        # (under TP the partial [T, H] is all-reduced first, so it is materialised)
        out = ops.linear(ops.linear_swiglu(h, lw["w_gate_up"]), lw["w_down"], defer=not self.tp.enabled)
        return self.tp.all_reduce_(out) if self.tp.enabled else out

    def _units(self):
        """(is_attention_half, layer, weights) for the halves this stage runs (whole halves only)."""
        for l in range(self.layer_start, self.layer_end):
            lw = self.layers[l - self.layer_start]
            if self.has(l, 0):
                yield True, l, lw
            if self.has(l, 3):
                yield False, l, lw

    @staticmethod
    def _dense(t):
        return t.materialize() if isinstance(t, ops.gemm.SplitKPartial) else t

    def _forward_llama(self, inp: torch.Tensor, meta: BatchMeta) -> torch.Tensor:
        cfg = self.cfg
        eps = cfg.norm_eps
        hs = cfg.hidden_size
        carry = None   # pending qkv / attention output / partial MLP sum handed over by a sub-layer cut
        if self.is_first:
            residual = ops.embedding(inp, self.embed["embed"])
        elif inp.shape[-1] > hs:
            # clone, not .contiguous(): a one-row column slice IS contiguous, and the residual is
            # updated in place -- a view would write into the caller's input (the decode graph's
            # static buffer, re-read by the capture warm-ups and the replay)
            residual = inp[:, :hs].clone(memory_format=torch.contiguous_format)
            carry = inp[:, hs:].clone(memory_format=torch.contiguous_format)
        else:
            residual = inp.clone()
        h = None   # output of the previous half, not yet added to the residual stream
        out_aux = None
        for l in range(self.layer_start, self.layer_end):
            lw = self.layers[l - self.layer_start]
            # ---- attention half: atoms 0 (norm + qkv), 1 (attention), 2 (o-projection)
            if self.has(l, 0) or self.has(l, 1) or self.has(l, 2):
                a = qkv = None
                if self.has(l, 0):
                    # W8A8 projection next (quant="fp8"): the norm kernel emits the per-token e4m3 input
                    q8 = isinstance(lw.get("wqkv"), ops.quant.Fp8Weight)
                    if h is None:
                        x = ops.rms_norm(residual, lw["attn_norm"], eps, quant_out=q8)
                    else:
                        x, residual = ops.fused_add_rms_norm(h, residual, lw["attn_norm"], eps, quant_out=q8)
                    h = None
                    qkv = ops.linear(x, lw["wqkv"], defer=knobs.K.defer_qkv and self.has(l, 1))
                    if not self.has(l, 1):
                        out_aux = self._dense(qkv)
                        break
                if self.has(l, 1):
                    a = self._attention(qkv if qkv is not None else carry, self.kv_index[l], meta)
                    if not self.has(l, 2):
                        out_aux = a
                        break
                if self.has(l, 2):
                    a = a if a is not None else carry
                    # defer: a split-K o-projection's reduce is fused into the MLP half's add + RMSNorm
                    # (TP: row-parallel partial sums, all-reduced over the group)
                    if self.tp.enabled:
                        h = self.tp.all_reduce_(ops.linear(a, lw["wo"]))
                    else:
                        h = ops.linear(a, lw["wo"], defer=knobs.K.defer_o)
            # ---- MLP half: atoms 3 / 4 (first / second half of the intermediate columns)
            if self.has(l, 3) or self.has(l, 4):
                q8 = isinstance(lw.get("w_gate_up"), ops.quant.Fp8Weight)
                if h is None:
                    x = ops.rms_norm(residual, lw["mlp_norm"], eps, quant_out=q8)
                else:
                    x, residual = ops.fused_add_rms_norm(h, residual, lw["mlp_norm"], eps, quant_out=q8)
                if self.has(l, 3) and self.has(l, 4):
                    h = self._mlp(x, lw)
                elif self.has(l, 3):                  # cut between the MLP halves: hand over the partial sum
                    out_aux = self._dense(self._mlp(x, lw))
                    h = None
                    break
                else:                                 # second half: add the first half's partial sum
                    h = ops.add_(self._dense(self._mlp(x, lw)), carry)
        if out_aux is not None:
            return torch.cat([residual, out_aux.view(out_aux.shape[0], -1)], dim=1)
        if not self.is_last:
            return ops.add_(residual, self._dense(h))
        return self._logits(h, residual, meta)

    def _logits(self, h, residual: torch.Tensor, meta: BatchMeta) -> torch.Tensor:
        # ``h`` may still be the last down projection's split-K partials: at decode (every row's
        # logits) they are reduced inside the final add + RMSNorm, as between layers
        cfg = self.cfg
        if meta.logits_idx is not None or cfg.arch == "gpt2":
            h = self._dense(h)
        if meta.logits_idx is not None:
            h = h.index_select(0, meta.logits_idx)
            residual = residual.index_select(0, meta.logits_idx)
        if cfg.arch == "gpt2":
            x = ops.layer_norm(h, self.head["final_norm"], self.head["final_norm_b"], cfg.norm_eps)
        else:
            x, _ = ops.fused_add_rms_norm(h, residual, self.head["final_norm"], cfg.norm_eps)
        return ops.linear(x, self.lm_head_weight())

    def _forward_gpt2(self, inp: torch.Tensor, meta: BatchMeta) -> torch.Tensor:
        cfg = self.cfg
        eps = cfg.norm_eps
        if self.is_first:
            x = ops.embedding(inp, self.embed["embed"])
            pe = ops.embedding(meta.positions, self.embed["pos_embed"])
            x = ops.add_(x, pe)
        else:
            x = inp.clone()
        for is_attn, l, lw in self._units():
            if is_attn:
                h = ops.layer_norm(x, lw["ln1_w"], lw["ln1_b"], eps)
                a = self._attention(ops.linear(h, lw["wqkv"], lw["bqkv"]), self.kv_index[l], meta)
                x = ops.add_(x, ops.linear(a, lw["wo"], lw["bo"]))
            else:
                h = ops.layer_norm(x, lw["ln2_w"], lw["ln2_b"], eps)
                f = ops.gelu_tanh(ops.linear(h, lw["w_fc"], lw["b_fc"]))
                x = ops.add_(x, ops.linear(f, lw["w_proj"], lw["b_proj"]))
        if not self.is_last:
            return x
        if meta.logits_idx is not None:
            x = x.index_select(0, meta.logits_idx)
        x = ops.layer_norm(x, self.head["final_norm"], self.head["final_norm_b"], eps)
        return ops.linear(x, self.lm_head_weight())
