"""Tensor parallelism inside a layer (Megatron-style column / row split) over RCCL.

Not in the reference ("TP ... out of scope for v1; if added: RCCL all-reduce").
Here it complements the layer pipeline for latency: a TP group of ``size`` ranks (one GPU
each) shares every layer of its stage:

  column-parallel   wqkv      rows of this rank's q heads | kv heads (GQA groups stay whole)
                    w_gate_up rows of this rank's slice of I, gate and up halves kept aligned
                    experts   (MoE) each expert's I sliced the same way; the router replicated
  expert-parallel   experts   (MoE, ``moe="ep"``) whole experts [r E/size, (r+1) E/size) per rank
                              instead: routing stays global (replicated router), a rank runs
                              only its experts' tokens, and the same all-reduce sums the group's
                              partial MoE outputs -- every expert GEMM at full I, ~T k / E rows
  row-parallel      wo        the matching q-head columns   -> partial [T, H] -> all-reduce
                    w_down    the matching I columns        -> partial [T, H] -> all-reduce
  vocab-parallel    lm_head   rows [r V/size, (r+1) V/size)  -> greedy: distributed argmax
  replicated        norms, embedding (every rank embeds its input ids itself)

Each rank's paged KV cache holds only its kv heads, so KV capacity grows with the group.
The two all-reduces per layer are RCCL collectives on the compute stream (bf16, [T, H]); on
MI355X's fully connected xGMI the ring is per-link bound (~153 GB/s), which is why TP is the
latency option (small batch, big model) and the pipeline the throughput one.

Driving a TP group: the leader runs the scheduler (an :class:`LLMEngine` with ``stage.tp`` set:
synchronous steps, eager launches) and broadcasts each step's packed ``HostBatch`` over the
group's gloo control group before executing it; followers (:func:`tp_follower_loop`) receive,
execute the same forward and join the same collectives.  Greedy tokens are bit-identical on every rank (the argmax
reduction is deterministic), so the leader needs nothing back.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, Optional

import numpy as np
import torch
import torch.distributed as dist

STOP = -1
ROUND_END = -2


@dataclass
class TPGroup:
    rank: int                 # rank within the TP group
    size: int
    group: object = None      # data collectives (RCCL on GPU, gloo on CPU)
    ctrl: object = None       # gloo: step metadata broadcast
    leader: int = 0           # global rank of the group's rank 0
    moe: str = "tp"           # MoE experts: "tp" = every expert's I sliced, "ep" = whole experts per rank

    @property
    def enabled(self) -> bool:
        return self.size > 1

    def expert_offset(self, num_experts: int) -> int:
        """First global expert this rank holds (expert parallel), else 0."""
        return self.rank * (num_experts // self.size) if self.moe == "ep" and self.size > 1 else 0

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            dist.all_reduce(t, group=self.group)
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        """[size, *t.shape] stacked in rank order."""
        out = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(out, t.contiguous(), group=self.group)
        return torch.stack(out)

    # ---- control: step metadata from the leader
    def bcast_meta(self, arr: Optional[np.ndarray]) -> np.ndarray:
        """Leader passes the packed int32 array, followers None; everyone gets it back."""
        n = torch.tensor([-1 if arr is None else arr.shape[0]], dtype=torch.int64)
        dist.broadcast(n, self.leader, group=self.ctrl)
        k = int(n.item())
        if k < 0:
            raise ValueError("bcast_meta: leader sent nothing")
        buf = torch.from_numpy(np.ascontiguousarray(arr, dtype=np.int32)) if self.rank == 0 \
            else torch.empty(k, dtype=torch.int32)
        dist.broadcast(buf, self.leader, group=self.ctrl)
        return buf.numpy()


# ------------------------------------------------------------------ weight sharding
def check_divisible(cfg, size: int, moe: str = "tp"):
    if size <= 1:
        return
    if moe not in ("tp", "ep"):
        raise ValueError(f"moe parallel mode {moe!r}: 'tp' or 'ep'")
    dims = [("num_heads", cfg.num_heads), ("num_kv_heads", cfg.num_kv_heads), ("vocab_size", cfg.vocab_size)]
    dims.append(("num_experts", cfg.num_experts) if cfg.is_moe and moe == "ep"
                else ("intermediate_size", cfg.intermediate_size))
    bad = [n for n, v in dims if v % size]
    if bad:
        raise ValueError(f"tensor parallel size {size} must divide {', '.join(bad)} of {cfg.name}")
    if cfg.arch == "gpt2":
        raise ValueError("tensor parallelism is implemented for the llama / mixtral families")


def shard_block(cfg, w: Dict[str, torch.Tensor], rank: int, size: int, moe: str = "tp") -> Dict[str, torch.Tensor]:
    """Full runtime block tensors -> this rank's shard (new contiguous tensors).  ``moe="ep"``:
    the MoE experts are split whole (expert parallelism) instead of sliced along I."""
    if size <= 1:
        return w
    d = cfg.head_dim
    hq, hkv = cfg.num_heads // size, cfg.num_kv_heads // size
    i_l = cfg.intermediate_size // size
    out = dict(w)
    qkv = w["wqkv"]
    q0 = rank * hq * d
    k0 = cfg.q_size + rank * hkv * d
    v0 = cfg.q_size + cfg.kv_size + rank * hkv * d
    out["wqkv"] = torch.cat([qkv[q0:q0 + hq * d], qkv[k0:k0 + hkv * d], qkv[v0:v0 + hkv * d]], 0).contiguous()
    out["wo"] = w["wo"][:, q0:q0 + hq * d].contiguous()
    i, a = cfg.intermediate_size, rank * i_l
    if cfg.is_moe and moe == "ep":
        e_l = cfg.num_experts // size
        # clone: a leading-dim slice is a contiguous VIEW, which would keep every expert resident
        out["experts_gate_up"] = w["experts_gate_up"][rank * e_l:(rank + 1) * e_l].clone()
        out["experts_down"] = w["experts_down"][rank * e_l:(rank + 1) * e_l].clone()
    elif cfg.is_moe:
        gu = w["experts_gate_up"]
        out["experts_gate_up"] = torch.cat([gu[:, a:a + i_l], gu[:, i + a:i + a + i_l]], 1).contiguous()
        out["experts_down"] = w["experts_down"][:, :, a:a + i_l].contiguous()
    else:
        gu = w["w_gate_up"]
        out["w_gate_up"] = torch.cat([gu[a:a + i_l], gu[i + a:i + a + i_l]], 0).contiguous()
        out["w_down"] = w["w_down"][:, a:a + i_l].contiguous()
    return out


def shard_vocab(t: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    if size <= 1:
        return t
    v = t.shape[0] // size
    return t[rank * v:(rank + 1) * v].clone()     # not a view: the full head must not stay resident


# ------------------------------------------------------------------ sampling over a vocab shard
def tp_sample(logits_local: torch.Tensor, tp: TPGroup, sampling_args: dict) -> torch.Tensor:
    """ids [B] int32 from vocab-sharded logits [B, V/size] -- identical on every rank.

    Greedy: each rank's local argmax (value, global index) is all-gathered and reduced with the
    same tie rule as the argmax kernel (largest value, then smallest index).  Otherwise the full
    logits are gathered and the leader's draw is broadcast (one sampler, one RNG stream)."""
    from ..engine.sampler import sample
    from .. import ops
    b, v_l = logits_local.shape
    if not sampling_args or all(t <= 0 for t in sampling_args.get("temperatures", [0.0])):
        idx = ops.argmax(logits_local).to(torch.int64)
        val = logits_local.gather(1, idx.unsqueeze(1)).squeeze(1).float()
        gidx = (idx + tp.rank * v_l).to(torch.float64)
        pairs = tp.all_gather(torch.stack([val.to(torch.float64), gidx], 1))       # [size, B, 2]
        vals, gids = pairs[..., 0], pairs[..., 1]
        best = vals.max(0).values
        cand = torch.where(vals == best.unsqueeze(0), gids, torch.full_like(gids, float("inf")))
        return cand.min(0).values.to(torch.int32)
    full = tp.all_gather(logits_local)                                             # [size, B, V_l]
    full = full.permute(1, 0, 2).reshape(b, tp.size * v_l)
    ids = sample(full, **sampling_args).to(torch.int32) if tp.rank == 0 else \
        torch.empty(b, dtype=torch.int32, device=full.device)
    dist.broadcast(ids, tp.leader, group=tp.group)
    return ids


def tp_follower_loop(runner, tp: TPGroup, stop_on_round_end: bool = True) -> str:
    """A tensor-parallel follower: run every step the leader broadcasts until STOP ("stop") or
    ROUND_END ("round")."""
    from ..engine.batch import HostBatch
    while True:
        arr = tp.bcast_meta(None)
        if arr.shape[0] == 1 and int(arr[0]) in (STOP, ROUND_END):
            if int(arr[0]) == STOP:
                return "stop"
            if stop_on_round_end:
                return "round"
            continue
        hb = HostBatch.unpack(arr.copy())
        logits = runner.execute(hb)
        tp_sample(logits, tp, hb.sampling_args())
