"""Host-side batch metadata construction and its (de)serialization.

A :class:`HostBatch` is the numpy form of one step's metadata; it is what stage 0
ships to the other pipeline stages (over the CPU control group) and what every stage
uploads into its :class:`BatchMeta` device tensors.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional

import numpy as np
import torch

from ..models.stage import BatchMeta
from .scheduler import Step

_FIELDS = ("ids", "positions", "slots", "seq_lens", "cu_seqlens", "block_tables", "logits_idx")


@dataclass
class HostBatch:
    is_prefill: bool
    ids: np.ndarray           # [T] int32
    positions: np.ndarray     # [T] int32
    slots: np.ndarray         # [T] int32
    seq_lens: np.ndarray      # [B] int32
    cu_seqlens: np.ndarray    # [B+1] int32
    block_tables: np.ndarray  # [B, MB] int32
    logits_idx: np.ndarray    # [B] int32
    max_q_len: int
    max_ctx: int
    slot: int = 0
    step_id: int = 0
    sampling: Optional[np.ndarray] = None   # [B, 3] int32: temperature*1e4, top_k, top_p*1e4 (None = greedy)
    # mixed prefill + decode step: the first num_decode sequences are single-token decode rows
    # (decode attention), the rest prefill chunks (prefill attention); 0 = not mixed
    num_decode: int = 0
    # the packed array this batch was unpacked from (its fields are views into it): pack() then
    # only refreshes the header instead of concatenating everything again
    raw: Optional[np.ndarray] = field(default=None, repr=False, compare=False)

    @property
    def num_tokens(self) -> int:
        return int(self.ids.shape[0])

    @property
    def num_seqs(self) -> int:
        return int(self.seq_lens.shape[0])

    # ------------------------------------------------------ wire format
    def pack(self) -> np.ndarray:
        """Flatten to one int32 array: [header(16) | fields...]."""
        if self.raw is not None:
            self.raw[6] = self.slot
            self.raw[7] = self.step_id
            return self.raw
        b, t = self.num_seqs, self.num_tokens
        mb = self.block_tables.shape[1] if self.block_tables.ndim == 2 else 0
        has_s = 1 if self.sampling is not None else 0
        hdr = np.array([1 if self.is_prefill else 0, t, b, mb, self.max_q_len, self.max_ctx, self.slot,
                        self.step_id, has_s, self.num_decode] + [0] * 6, dtype=np.int32)
        parts = [hdr, self.ids, self.positions, self.slots, self.seq_lens, self.cu_seqlens,
                 self.block_tables.reshape(-1), self.logits_idx]
        if has_s:
            parts.append(self.sampling.reshape(-1))
        return np.concatenate([p.astype(np.int32, copy=False).reshape(-1) for p in parts])

    def sampling_args(self) -> dict:
        if self.sampling is None:
            return {}
        s = self.sampling
        return {"temperatures": (s[:, 0] / 1e4).tolist(), "top_k": s[:, 1].tolist(),
                "top_p": (s[:, 2] / 1e4).tolist()}

    @staticmethod
    def unpack(arr: np.ndarray) -> "HostBatch":
        hdr = arr[:16]
        pf, t, b, mb, mq, mc, slot, sid, has_s, nd = (int(x) for x in hdr[:10])
        o = 16
        def take(n):
            nonlocal o
            v = arr[o:o + n]
            o += n
            return v
        ids, pos, slots = take(t), take(t), take(t)
        seq_lens, cu = take(b), take(b + 1)
        bt = take(b * mb).reshape(b, mb)
        lidx = take(b)
        samp = take(3 * b).reshape(b, 3) if has_s else None
        return HostBatch(bool(pf), ids, pos, slots, seq_lens, cu, bt, lidx, mq, mc, slot, sid, samp, raw=arr,
                         num_decode=nd)


def next_pow2(x: int, lo: int = 1) -> int:
    p = lo
    while p < x:
        p *= 2
    return p


def build_host_batch(step: Step, bm, block_size: int, max_blocks: Optional[int] = None,
                     step_id: int = 0) -> HostBatch:
    """Metadata of one step.  Decode steps of the native batcher arrive packed already (their
    block-table width is the scheduler's ``max_blocks``); only the step id is stamped here.  A
    mixed step is the decode rows' packed batch followed by its prefill chunk's (merge_mixed)."""
    if getattr(step, "mixed", False):
        dec = HostBatch.unpack(step.packed)
        pre = build_host_batch(Step(True, step.seqs, step.slot), bm, block_size, None, step_id)
        return merge_mixed(dec, pre, step.slot, step_id)
    if step.packed is not None:
        step.packed[7] = step_id
        return HostBatch.unpack(step.packed)
    seqs = step.seqs
    b = len(seqs)
    seq_ids = np.fromiter((s.seq_id for s in seqs), dtype=np.int64, count=b)
    if step.is_prefill:
        # chunked prefill: a sequence computes [num_cached, num_cached + prefill_len) and attends to
        # everything before it already in the KV cache (seq_lens = context after this step)
        starts = np.fromiter((s.num_cached for s in seqs), dtype=np.int32, count=b)
        qlens = np.fromiter((s.prefill_len for s in seqs), dtype=np.int32, count=b)
        seq_lens = starts + qlens
        cu = np.zeros(b + 1, dtype=np.int32)
        np.cumsum(qlens, out=cu[1:])
        t = int(cu[-1])
        ids = np.empty(t, dtype=np.int32)
        positions = np.empty(t, dtype=np.int32)
        for i, s in enumerate(seqs):
            toks = s.all_tokens()
            a, e = s.num_cached, s.num_cached + int(qlens[i])
            ids[cu[i]:cu[i + 1]] = toks[a:e]
            positions[cu[i]:cu[i + 1]] = np.arange(a, e, dtype=np.int32)
        logits_idx = (cu[1:] - 1).astype(np.int32)
        max_q_len = int(qlens.max()) if b else 0
    else:
        seq_lens = np.fromiter((s.total_len for s in seqs), dtype=np.int32, count=b)
        starts = seq_lens - 1
        qlens = np.ones(b, dtype=np.int32)
        cu = np.arange(b + 1, dtype=np.int32)
        ids = np.fromiter((s.last_token() for s in seqs), dtype=np.int32, count=b)
        positions = starts.astype(np.int32)
        logits_idx = np.arange(b, dtype=np.int32)
        max_q_len = 1
    t = ids.shape[0]
    slots = np.empty(t, dtype=np.int32)
    n = bm.fill_slots(seq_ids, starts.astype(np.int32), qlens.astype(np.int32), slots)
    assert n == t
    need_blocks = int(-(-int(seq_lens.max()) // block_size)) if b else 1
    mb = max_blocks if max_blocks is not None else need_blocks
    if mb < need_blocks:
        raise ValueError("max_blocks too small for batch")
    bt = np.zeros((b, mb), dtype=np.int32)
    bm.fill_block_tables(seq_ids, bt, 0)
    max_ctx = int(seq_lens.max()) if b else 0
    sampling = None
    if any(s.params.temperature > 0 for s in seqs):
        sampling = np.array([[int(round(s.params.temperature * 1e4)), int(s.params.top_k),
                              int(round(s.params.top_p * 1e4))] for s in seqs], dtype=np.int32)
    return HostBatch(step.is_prefill, ids, positions, slots, seq_lens, cu, bt, logits_idx, max_q_len,
                     max_ctx, step.slot, step_id, sampling)


def merge_mixed(dec: HostBatch, pre: HostBatch, slot: int, step_id: int) -> HostBatch:
    """One HostBatch for a mixed step: decode rows (one token each) first, then the prefill
    chunks; block tables padded to the wider of the two; runs the eager prefill path with
    ``num_decode`` telling the attention which rows are decode rows."""
    nd = dec.num_seqs
    mb = max(dec.block_tables.shape[1], pre.block_tables.shape[1])
    bt = np.zeros((nd + pre.num_seqs, mb), dtype=np.int32)
    bt[:nd, : dec.block_tables.shape[1]] = dec.block_tables
    bt[nd:, : pre.block_tables.shape[1]] = pre.block_tables
    cu = np.concatenate([np.arange(nd, dtype=np.int32), pre.cu_seqlens.astype(np.int32) + nd])
    sampling = None
    if dec.sampling is not None or pre.sampling is not None:
        zd = np.zeros((nd, 3), np.int32)
        zp = np.zeros((pre.num_seqs, 3), np.int32)
        sampling = np.concatenate([dec.sampling if dec.sampling is not None else zd,
                                   pre.sampling if pre.sampling is not None else zp])
    return HostBatch(True, np.concatenate([dec.ids, pre.ids]).astype(np.int32),
                     np.concatenate([dec.positions, pre.positions]).astype(np.int32),
                     np.concatenate([dec.slots, pre.slots]).astype(np.int32),
                     np.concatenate([dec.seq_lens, pre.seq_lens]).astype(np.int32), cu, bt,
                     np.concatenate([np.arange(nd, dtype=np.int32), pre.logits_idx.astype(np.int32) + nd]),
                     max(1, pre.max_q_len), max(dec.max_ctx, pre.max_ctx), slot, step_id, sampling, num_decode=nd)


def build_decode_batch(seq_ids: np.ndarray, seq_lens: np.ndarray, bm, block_size: int, max_blocks: int,
                       step_id: int = 0, slot: int = 0) -> HostBatch:
    """Decode HostBatch straight from arrays (lookahead path: the input ids are not known on the
    host yet -- they are gathered on the device -- so ``ids`` is a zero placeholder)."""
    b = seq_ids.shape[0]
    positions = (seq_lens - 1).astype(np.int32)
    slots = np.empty(b, dtype=np.int32)
    n = bm.fill_slots(seq_ids, positions, np.ones(b, dtype=np.int32), slots)
    assert n == b
    need_blocks = int(-(-int(seq_lens.max()) // block_size)) if b else 1
    if max_blocks < need_blocks:
        raise ValueError("max_blocks too small for batch")
    bt = np.zeros((b, max_blocks), dtype=np.int32)
    bm.fill_block_tables(seq_ids, bt, 0)
    return HostBatch(False, np.zeros(b, dtype=np.int32), positions, slots, seq_lens.astype(np.int32),
                     np.arange(b + 1, dtype=np.int32), bt, np.arange(b, dtype=np.int32), 1,
                     int(seq_lens.max()) if b else 0, slot, step_id, None)


def to_device_meta(hb: HostBatch, device, pad_ctx_to: Optional[int] = None) -> (torch.Tensor, BatchMeta):
    """Upload a HostBatch; returns (ids tensor, BatchMeta)."""
    dev = torch.device(device)
    nb = dev.type == "cuda"
    def up(a, dtype=torch.int32):
        t = torch.from_numpy(np.ascontiguousarray(a))
        if nb:
            t = t.pin_memory()
        return t.to(dev, dtype=dtype, non_blocking=nb)
    ids = up(hb.ids)
    meta = BatchMeta(
        is_prefill=hb.is_prefill, positions=up(hb.positions), slot_mapping=up(hb.slots),
        block_tables=up(hb.block_tables), seq_lens=up(hb.seq_lens),
        cu_seqlens_q=up(hb.cu_seqlens) if hb.is_prefill else None,
        logits_idx=up(hb.logits_idx, torch.int64) if hb.is_prefill else None,
        max_q_len=hb.max_q_len, max_ctx=pad_ctx_to or hb.max_ctx, num_seqs=hb.num_seqs,
        num_tokens=hb.num_tokens)
    nd = hb.num_decode
    if nd and hb.is_prefill:
        # mixed step: the prefill rows' own cu_seqlens (from 0) and the decode rows' context bound
        meta.num_decode = nd
        meta.cu_seqlens_p = up(hb.cu_seqlens[nd:] - nd)
        meta.max_ctx_d = int(hb.seq_lens[:nd].max())
        meta.max_q_len_p = int((hb.cu_seqlens[nd + 1:] - hb.cu_seqlens[nd:-1]).max())
    return ids, meta
