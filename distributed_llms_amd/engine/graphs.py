"""HIP-graph capture/replay of the per-stage decode step (N5 in SURVEY §2.2).

A decode step of an 8B model is ~300 kernel launches; eager launch costs ~3-4 us
each on the host, so the step is captured once per (batch bucket, context bucket) and
replayed.  Inputs are copied into persistent device buffers; padded rows of a bucket
write their K/V into the reserved scratch block 0 (slot 0) and attend to one token,
so they never touch a live sequence.
"""
from __future__ import annotations

import threading
from typing import Dict, Optional, Tuple

import torch

from ..models.stage import BatchMeta, ModelStage
from .batch import HostBatch, next_pow2

SCRATCH_SEQ_ID = -1      # owns block 0 in the BlockManager
_CAPTURE_LOCK = threading.Lock()   # one graph capture at a time per process


class DecodeGraphRunner:
    def __init__(self, stage: ModelStage, max_batch: int, max_blocks: int, batch_sizes,
                 min_ctx_bucket: int = 256):
        self.stage = stage
        self.dev = stage.device
        self.max_batch = max(batch_sizes) if batch_sizes else max_batch
        self.max_batch = max(self.max_batch, 1)
        self.max_blocks = max_blocks
        self.block_size = stage.kv.block_size
        self.batch_sizes = sorted(set(b for b in batch_sizes if b <= self.max_batch)) or [self.max_batch]
        self.min_ctx_bucket = min_ctx_bucket
        cfg = stage.cfg
        mb, dev = self.max_batch, self.dev
        # every int32 graph input lives in ONE device buffer laid out like the pinned staging
        # buffer -- [ids | positions | slots | seq_lens] x max_batch, then the block table rows --
        # so a step's inputs go up in a single H2D copy (the first 4 * max_batch + bb * max_blocks
        # ints) instead of five
        self.dev_in = torch.zeros(4 * mb + mb * max_blocks, dtype=torch.int32, device=dev)
        self.ids = self.dev_in[0:mb]
        self.positions = self.dev_in[mb:2 * mb]
        self.slots = self.dev_in[2 * mb:3 * mb]
        self.seq_lens = self.dev_in[3 * mb:4 * mb]
        self.seq_lens.fill_(1)
        self.block_tables = self.dev_in[4 * mb:].view(mb, max_blocks)
        self.hidden = None if stage.is_first else torch.zeros(mb, stage.in_width, dtype=stage.dtype, device=dev)
        max_splits = 64
        self.ws = (torch.empty(mb * cfg.num_heads * max_splits * cfg.head_dim, dtype=torch.float32, device=dev),
                   torch.empty(mb * cfg.num_heads * max_splits * 2, dtype=torch.float32, device=dev))
        self.pinned = torch.empty(4 * mb + mb * max_blocks, dtype=torch.int32).pin_memory()
        self.pinned_np = self.pinned.numpy()
        self.graphs: Dict[Tuple[int, int], Tuple[torch.cuda.CUDAGraph, torch.Tensor]] = {}
        self.pool = None
        self.copy_done: Optional[torch.cuda.Event] = None
        self.capture_stream: Optional[torch.cuda.Stream] = None

    def bucket(self, b: int, max_ctx: int) -> Tuple[int, int]:
        bb = next(x for x in self.batch_sizes if x >= b)
        cb = min(next_pow2(max_ctx, self.min_ctx_bucket), self.max_blocks * self.block_size)
        return bb, cb

    def can_run(self, b: int, max_ctx: int) -> bool:
        return b <= self.max_batch and max_ctx <= self.max_blocks * self.block_size

    def _meta(self, bb: int, cb: int) -> BatchMeta:
        return BatchMeta(is_prefill=False, positions=self.positions[:bb], slot_mapping=self.slots[:bb],
                         block_tables=self.block_tables[:bb], seq_lens=self.seq_lens[:bb], max_q_len=1,
                         max_ctx=cb, num_seqs=bb, num_tokens=bb, attn_workspace=self.ws)

    def _inp(self, bb: int) -> torch.Tensor:
        return self.ids[:bb] if self.stage.is_first else self.hidden[:bb]

    def capture(self, bb: int, cb: int):
        with _CAPTURE_LOCK:
            return self._capture(bb, cb)

    def _capture(self, bb: int, cb: int):
        meta = self._meta(bb, cb)
        # warm up outside capture (allocator, lazy module init)
        if self.capture_stream is None:
            self.capture_stream = torch.cuda.Stream(self.dev)
        s = self.capture_stream
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self.stage.forward(self._inp(bb), meta)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        # own capture stream: per-stream GEMM workspaces stay private to this runner's graphs;
        # thread_local mode: RCCL/gloo threads of this process may keep calling HIP meanwhile
        with torch.cuda.graph(g, pool=self.pool, stream=s, capture_error_mode="thread_local"):
            out = self.stage.forward(self._inp(bb), meta)
        self.graphs[(bb, cb)] = (g, out)
        return g, out

    def load_inputs(self, hb: HostBatch, bb: int, hidden: Optional[torch.Tensor] = None):
        b = hb.num_seqs
        mbk = hb.block_tables.shape[1]
        if mbk > self.max_blocks:
            raise ValueError("block table wider than graph buffers")
        if self.copy_done is not None:
            self.copy_done.synchronize()   # previous step's H2D may still read the pinned buffer
        # numpy views of the pinned staging buffer: a handful of memcpy-sized writes per step
        # instead of one torch op (~5-10 us of host time each) per field
        n, mb, w = bb, self.max_batch, self.max_blocks
        p = self.pinned_np
        pv = p[: 4 * mb].reshape(4, mb)
        pv[0, :b] = hb.ids
        pv[1, :b] = hb.positions
        pv[2, :b] = hb.slots
        pv[3, :b] = hb.seq_lens
        if n > b:                                       # padded rows: scratch slot 0, one token
            pv[:3, b:n] = 0
            pv[3, b:n] = 1
        bt = p[4 * mb: 4 * mb + n * w].reshape(n, w)
        bt[:b, :mbk] = hb.block_tables
        bt[:b, mbk:] = 0
        bt[b:] = 0
        cnt = 4 * mb + n * w
        self.dev_in[:cnt].copy_(self.pinned[:cnt], non_blocking=True)
        if self.copy_done is None:
            self.copy_done = torch.cuda.Event()
        self.copy_done.record()
        if hidden is not None:
            self.hidden[:b].copy_(hidden[:b])
            if bb > b:
                self.hidden[b:bb].zero_()

    def run(self, hb: HostBatch, hidden: Optional[torch.Tensor] = None,
            ids_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Replay the bucket's graph; returns the (static) output truncated to the real batch.
        ``ids_dev``: device-resident input ids overriding ``hb.ids`` (lookahead decode)."""
        b = hb.num_seqs
        bb, cb = self.bucket(b, hb.max_ctx)
        self.load_inputs(hb, bb, hidden)
        if ids_dev is not None:
            self.ids[:b].copy_(ids_dev, non_blocking=True)
        entry = self.graphs.get((bb, cb))
        if entry is None:
            entry = self.capture(bb, cb)
        g, out = entry
        g.replay()
        return out[:b]
