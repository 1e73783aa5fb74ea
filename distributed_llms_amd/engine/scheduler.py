"""Continuous-batching request scheduler with pipeline microbatch slots.

Replaces the reference's FIFO ``task_queue`` + broadcast (``src/master/node.py:227-277``)
and its busy-polled ``result_queue`` (D17).  Sequences are bound to one of
``num_slots`` microbatch slots (slots = pipeline stages, so every stage has a
microbatch in flight); each call to :meth:`schedule` for a slot returns either a
prefill step (admitting waiting requests, bounded by ``max_prefill_tokens`` and free KV
blocks) or a decode step over the slot's running sequences.  KV blocks come from the
native :class:`BlockManager`; when a decode step cannot grow a sequence the youngest
running sequence of that slot is preempted (blocks freed, recomputed later).
"""
from __future__ import annotations

import collections
import time
from dataclasses import dataclass
from typing import Deque, Dict, List, Optional

import numpy as np

from .sequence import Sequence, SeqStatus


@dataclass
class Step:
    is_prefill: bool
    seqs: List[Sequence]
    slot: int = 0

    @property
    def num_tokens(self) -> int:
        if self.is_prefill:
            return sum(s.total_len - s.num_cached for s in self.seqs)
        return len(self.seqs)


class Scheduler:
    def __init__(self, block_manager, num_slots: int = 1, max_batch: int = 256,
                 max_prefill_tokens: int = 16384, max_seq_len: int = 4096):
        self.bm = block_manager
        self.num_slots = max(1, num_slots)
        self.max_batch = max_batch
        self.max_prefill_tokens = max_prefill_tokens
        self.max_seq_len = max_seq_len
        self.waiting: Deque[Sequence] = collections.deque()
        self.running: List[List[Sequence]] = [[] for _ in range(self.num_slots)]
        self.finished: List[Sequence] = []
        self.num_preemptions = 0

    # ------------------------------------------------------------ requests
    def add(self, seq: Sequence) -> None:
        if len(seq.prompt) + 1 > self.max_seq_len:
            seq.finish("too_long")
            self.finished.append(seq)
            return
        seq.status = SeqStatus.WAITING
        self.waiting.append(seq)

    def abort(self, seq_id: int) -> bool:
        for s in list(self.waiting):
            if s.seq_id == seq_id:
                self.waiting.remove(s)
                s.finish("abort")
                self.finished.append(s)
                return True
        for run in self.running:
            for s in run:
                if s.seq_id == seq_id:
                    run.remove(s)
                    self.bm.free_sequence(s.seq_id)
                    s.finish("abort")
                    self.finished.append(s)
                    return True
        return False

    def has_work(self) -> bool:
        return bool(self.waiting) or any(self.running)

    def num_running(self) -> int:
        return sum(len(r) for r in self.running)

    def _pick_slot_for_admission(self, slot: int) -> bool:
        """Admit into `slot` only if it is (one of) the least-loaded slots."""
        n = len(self.running[slot])
        return n <= min(len(r) for r in self.running)

    # ------------------------------------------------------------ schedule
    def schedule(self, slot: int = 0) -> Optional[Step]:
        running = self.running[slot]
        admitted: List[Sequence] = []
        if self.waiting and self._pick_slot_for_admission(slot):
            tokens = 0
            per_slot_cap = self.max_batch
            while self.waiting and len(running) + len(admitted) < per_slot_cap:
                seq = self.waiting[0]
                n = seq.total_len - seq.num_cached
                if admitted and tokens + n > self.max_prefill_tokens:
                    break
                if not self.bm.ensure_capacity(seq.seq_id, seq.total_len):
                    break
                self.waiting.popleft()
                seq.status = SeqStatus.RUNNING
                seq.slot = slot
                admitted.append(seq)
                tokens += n
            if admitted:
                return Step(True, admitted, slot)
        if not running:
            return None
        # decode: every running sequence of the slot needs room for one more token (one native
        # call for the whole slot; on failure preempt the youngest and retry from there)
        i = 0
        while i < len(running):
            rest = running[i:]
            ids = np.fromiter((s.seq_id for s in rest), dtype=np.int64, count=len(rest))
            lens = np.fromiter((len(s.prompt) + len(s.output) for s in rest), dtype=np.int64, count=len(rest))
            bad = self.bm.ensure_capacity_batch(ids, lens)
            if bad < 0:
                break
            i += bad
            victim = running.pop()  # youngest
            self._preempt(victim)
        if not running:
            return None
        return Step(False, list(running), slot)

    def _preempt(self, seq: Sequence):
        self.bm.free_sequence(seq.seq_id)
        seq.num_cached = 0
        seq.status = SeqStatus.WAITING
        self.waiting.appendleft(seq)
        self.num_preemptions += 1

    # ------------------------------------------------------------ results
    def complete(self, step: Step, tokens, now: Optional[float] = None) -> List[Sequence]:
        """Apply sampled tokens of an executed step; returns sequences that finished."""
        done = []
        running = self.running[step.slot]
        if hasattr(tokens, "tolist"):
            tokens = tokens.tolist()      # python ints once, not a numpy scalar per sequence
        now = time.perf_counter() if now is None else now
        prefill = step.is_prefill
        for seq, tok in zip(step.seqs, tokens):
            st = seq.status
            if st is SeqStatus.FINISHED or st is SeqStatus.ABORTED:   # aborted while in flight
                continue
            seq.num_cached = len(seq.prompt) + len(seq.output)
            if prefill:
                running.append(seq)
            if seq.append(tok, now) or seq.num_cached + 1 >= self.max_seq_len:
                if not seq.finished:
                    seq.finish("max_seq_len", now)
                if seq in running:
                    running.remove(seq)
                self.bm.free_sequence(seq.seq_id)
                self.finished.append(seq)
                done.append(seq)
        return done

    def pop_finished(self) -> List[Sequence]:
        f, self.finished = self.finished, []
        return f
