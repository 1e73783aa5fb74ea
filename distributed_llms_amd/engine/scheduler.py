"""Continuous-batching request scheduler with pipeline microbatch slots.

Replaces the reference's FIFO ``task_queue`` + broadcast (``src/master/node.py:227-277``)
and its busy-polled ``result_queue`` (D17).  Sequences are bound to one of
``num_slots`` microbatch slots (slots = pipeline stages, so every stage has a
microbatch in flight); each call to :meth:`schedule` for a slot returns either a
prefill step (admitting waiting requests, bounded by ``max_prefill_tokens`` and free KV
blocks) or a decode step over the slot's running sequences.  KV blocks come from the
native :class:`BlockManager`; when a decode step cannot grow a sequence the youngest
running sequence of that slot is preempted (blocks freed, recomputed later).  The decode
bookkeeping is native (csrc/runtime/slot_batcher.cpp): at batch 256 a decode microbatch costs
the driver two C++ calls instead of ~0.9 ms of per-sequence Python (bench/host_overhead.py).
"""
from __future__ import annotations

import collections
import time
from typing import Deque, Dict, List, Optional

import numpy as np

from .. import _ext
from .sequence import Sequence, SeqStatus


class Step:
    """One microbatch: a prefill over ``seqs`` or a decode step.  Decode steps from the native
    batcher carry their sequence ids (``rows``), the packed batch metadata (``packed``, the
    HostBatch wire format) and, for lookahead steps, ``keep`` (positions of the rows in the slot's
    previous step); ``seqs`` is then resolved lazily from the scheduler's registry.

    A MIXED step (``mixed``; ``is_prefill`` is True: it runs the eager prefill path) carries both:
    the slot's decode rows (``rows`` / ``packed``, one token each, first in the batch) and a bounded
    prefill chunk over ``seqs``."""

    __slots__ = ("is_prefill", "_seqs", "slot", "rows", "packed", "keep", "_live", "mixed")

    def __init__(self, is_prefill: bool, seqs: Optional[List[Sequence]] = None, slot: int = 0,
                 rows: Optional[np.ndarray] = None, packed: Optional[np.ndarray] = None,
                 keep: Optional[np.ndarray] = None, live: Optional[Dict[int, Sequence]] = None,
                 mixed: bool = False):
        self.is_prefill = is_prefill
        self._seqs = seqs
        self.slot = slot
        self.rows = rows
        self.packed = packed
        self.keep = keep
        self._live = live
        self.mixed = mixed

    @property
    def seqs(self) -> List[Sequence]:
        """The step's sequences (a mixed step: its PREFILL sequences; see decode_seqs)."""
        if self._seqs is None:
            live = self._live
            self._seqs = [live[int(i)] for i in self.rows]
        return self._seqs

    @property
    def decode_seqs(self) -> List[Sequence]:
        """A mixed step's decode sequences (in row order)."""
        return [self._live[int(i)] for i in self.rows] if self.mixed else []

    @property
    def num_decode(self) -> int:
        return len(self.rows) if self.mixed else 0

    @property
    def size(self) -> int:
        """Sequences (= logit rows) in the step."""
        if self.mixed:
            return len(self.rows) + len(self._seqs)
        return len(self.rows) if self.rows is not None else len(self._seqs)

    @property
    def num_tokens(self) -> int:
        if self.mixed:
            return len(self.rows) + sum(s.prefill_len for s in self._seqs)
        if self.is_prefill:
            return sum(s.prefill_len for s in self.seqs)
        return self.size


def _eos_of(seq: Sequence) -> int:
    return -1 if (seq.params.ignore_eos or seq.eos_token_id is None) else int(seq.eos_token_id)


class Scheduler:
    """Admission (prefill, chunked for prompts longer than the step's token budget) is
    per-sequence Python; the running decode set of every slot lives in
    the native :class:`SlotBatcher` (csrc/runtime/slot_batcher.cpp), which builds each decode
    step's packed metadata and applies its sampled tokens in one call each.  A running sequence's
    Python ``output`` list is brought up to date when it leaves the running set (finish,
    preemption, abort); :meth:`sync_output` refreshes it earlier on demand."""

    MIN_CHUNK = 32          # smallest chunk worth starting in a step whose budget is nearly used

    def __init__(self, block_manager, num_slots: int = 1, max_batch: int = 256,
                 max_prefill_tokens: int = 16384, max_seq_len: int = 4096, mixed_prefill_tokens: int = 0):
        """``mixed_prefill_tokens`` > 0: a slot with running sequences admits waiting prompts as a
        chunk of at most this many tokens (capped by ``max_prefill_tokens``) riding along with its
        decode rows (a mixed step) instead of a prefill-only step that stalls every running
        sequence for a whole chunk.  Large budgets keep a burst's admission as fast as
        prefill-first (the decode rows ride along for free); small ones bound the inter-token
        latency of the running rows."""
        self.bm = block_manager
        self.num_slots = max(1, num_slots)
        self.max_batch = max_batch
        self.max_prefill_tokens = max_prefill_tokens
        self.mixed_prefill_tokens = min(max(0, int(mixed_prefill_tokens)), max_prefill_tokens)
        self.num_mixed = 0
        self.max_seq_len = max_seq_len
        self.max_blocks = -(-max_seq_len // block_manager.block_size)    # decode block-table width
        self.native = _ext.runtime().SlotBatcher(block_manager, self.num_slots, max_seq_len)
        self.live: Dict[int, Sequence] = {}          # sequences registered with the native batcher
        self.waiting: Deque[Sequence] = collections.deque()
        self.finished: List[Sequence] = []
        self.num_preemptions = 0
        self.num_prefilling = 0                       # admitted, prefill step not completed yet

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
                self.bm.free_sequence(s.seq_id)       # a partly prefilled prompt holds blocks
                s.finish("abort")
                self.finished.append(s)
                return True
        if seq_id in self.live and self.native.abort(seq_id):
            self._sync_finished(time.perf_counter())
            return True
        return False

    def has_work(self) -> bool:
        return bool(self.waiting) or self.native.num_running_total() > 0

    def num_running(self) -> int:
        return self.native.num_running_total()

    @property
    def running(self) -> List[List[Sequence]]:
        """Running sequences per slot, oldest first (a snapshot)."""
        return [[self.live[int(i)] for i in self.native.running_ids(s)] for s in range(self.num_slots)]

    def sync_output(self, seq: Sequence) -> List[int]:
        """Generated ids of ``seq`` so far, including those still held by the native batcher."""
        if seq.seq_id in self.live and not seq.finished:
            return seq.output + self.native.peek_output(seq.seq_id).tolist()
        return list(seq.output)

    def _admission_target(self) -> int:
        """Sequences a slot should hold: an even share of everything admitted or waiting (capped by
        max_batch).  Each slot tops itself up to it when its turn comes, so a burst of requests is
        prefilled in full-size chunks on every slot at once and decode starts at full batch,
        instead of least-loaded-first admission starting some slots' decode with a quarter of
        their rows while the others still prefill."""
        total = self.native.num_running_total() + self.num_prefilling + len(self.waiting)
        return min(self.max_batch, -(-total // self.num_slots))

    # ------------------------------------------------------------ schedule
    def _admit(self, slot: int, n_running: int, max_tokens: int):
        """Admit waiting prompts (whole, or a chunk of the first one that does not fit) into a step
        of at most ``max_tokens`` prompt tokens.  Returns (admitted, blocked on KV)."""
        admitted: List[Sequence] = []
        tokens = 0
        target = self._admission_target()
        blocked = False
        while self.waiting and n_running + len(admitted) < target:
            seq = self.waiting[0]
            n = seq.total_len - seq.num_cached
            budget = max_tokens - tokens
            if n > budget:
                # chunked prefill: a prompt longer than what is left of this step's token
                # budget contributes a chunk; the rest follows in later steps
                if admitted and budget < min(n, self.MIN_CHUNK):
                    break
                if budget <= 0:
                    break
                n = budget
            seq.chunk = n if n < seq.total_len - seq.num_cached else 0
            if not self.bm.ensure_capacity(seq.seq_id, seq.num_cached + n):
                seq.chunk = 0
                blocked = True
                break
            self.waiting.popleft()
            seq.status = SeqStatus.RUNNING
            seq.slot = slot
            admitted.append(seq)
            tokens += n
        return admitted, blocked

    def schedule(self, slot: int = 0, _retry: bool = True) -> Optional[Step]:
        n_running = self.native.num_running(slot)
        if self.waiting and n_running and self.mixed_prefill_tokens:
            # mixed step: the slot's decode rows first (they get KV before any new prompt), then a
            # bounded chunk of waiting prompts in the same forward
            res = self.native.build_decode(slot, self.max_blocks, 0, False)
            self._sync_preempted()
            if res is not None:
                packed, rows, _ = res
                # one token budget per step (decode rows + prompt tokens <= max_prefill_tokens): the
                # step's activations fit every buffer sized for a prefill step (pipeline hop slots)
                budget = min(self.mixed_prefill_tokens, self.max_prefill_tokens - len(rows))
                admitted, _blocked = self._admit(slot, len(rows), budget) if budget > 0 else ([], False)
                if admitted:
                    self.num_prefilling += len(admitted)
                    self.num_mixed += 1
                    return Step(True, admitted, slot, rows=rows, packed=packed, live=self.live, mixed=True)
                return Step(False, None, slot, rows=rows, packed=packed, live=self.live)
            n_running = self.native.num_running(slot)
        if self.waiting:
            admitted, blocked = self._admit(slot, n_running, self.max_prefill_tokens)
            if admitted:
                self.num_prefilling += len(admitted)
                return Step(True, admitted, slot)
            if blocked and _retry and self._break_kv_deadlock():
                return self.schedule(slot, _retry=False)
        if not n_running:
            return None
        # decode: every running sequence of the slot needs room for one more token; on failure
        # the native batcher preempts the youngest until the rest fits
        res = self.native.build_decode(slot, self.max_blocks, 0, False)
        self._sync_preempted()
        if res is None:
            return None
        packed, rows, _ = res
        return Step(False, None, slot, rows=rows, packed=packed, live=self.live)

    def _break_kv_deadlock(self) -> bool:
        """The head of the queue cannot get KV blocks.  While anything runs or a prefill is in
        flight, blocks will come back (finishes, preemption); when nothing does, the only holders
        are partly prefilled prompts still waiting for their next chunk, and none of them can
        advance -- e.g. two long prompts on two slots each holding half of a small pool.  Drop
        the cached chunks of every waiting prompt but the head (they are recomputed later); if
        the head alone still cannot fit an otherwise empty pool, it never will: finish it.
        Returns True when the queue changed (the caller retries once)."""
        if self.native.num_running_total() > 0 or self.num_prefilling > 0 or not self.waiting:
            return False
        head = self.waiting[0]
        freed = False
        for s in list(self.waiting)[1:]:
            if s.num_cached > 0:
                self.bm.free_sequence(s.seq_id)
                s.num_cached = 0
                s.chunk = 0
                freed = True
        if freed:
            return True
        # nothing else holds blocks: the pool cannot hold the head's next chunk at all
        self.waiting.popleft()
        self.bm.free_sequence(head.seq_id)
        head.finish("kv_capacity")
        self.finished.append(head)
        return True

    def schedule_lookahead(self, slot: int) -> Optional[Step]:
        """The slot's next decode step, built while its newest decode step is still in flight
        (input ids come from the device).  None when the host must catch up first."""
        if self.waiting:
            return None
        res = self.native.build_decode(slot, self.max_blocks, 0, True)
        if res is None:
            return None
        packed, rows, keep = res
        return Step(False, None, slot, rows=rows, packed=packed, keep=keep, live=self.live)

    def _sync_preempted(self):
        for sid in self.native.take_preempted():
            seq = self.live.pop(int(sid))
            toks, times = self.native.take_output(sid)
            seq.output.extend(toks.tolist())
            seq.token_times.extend(times.tolist())
            seq.num_cached = 0
            seq.status = SeqStatus.WAITING
            self.waiting.appendleft(seq)
            self.num_preemptions += 1

    def _sync_finished(self, now: float) -> List[Sequence]:
        done = []
        for sid, reason in self.native.take_finished():
            seq = self.live.pop(int(sid))
            toks, times = self.native.take_output(sid)
            seq.output.extend(toks.tolist())
            seq.token_times.extend(times.tolist())
            seq.finish(reason, float(times[-1]) if len(times) else now)
            self.finished.append(seq)
            done.append(seq)
        return done

    # ------------------------------------------------------------ results
    def complete(self, step: Step, tokens, now: Optional[float] = None) -> List[Sequence]:
        """Apply sampled tokens of an executed step; returns sequences that finished."""
        now = time.perf_counter() if now is None else now
        if not step.is_prefill:
            toks = np.asarray(tokens, dtype=np.int32)
            if self.native.complete(step.slot, step.rows, toks, now):
                return self._sync_finished(now)
            return []
        done = []
        if step.mixed:
            # decode rows first in the batch: their tokens go to the native batcher
            toks = np.asarray(tokens, dtype=np.int32)
            nd = len(step.rows)
            if self.native.complete(step.slot, step.rows, np.ascontiguousarray(toks[:nd]), now):
                done.extend(self._sync_finished(now))
            tokens = toks[nd:]
        self.num_prefilling -= len(step.seqs)
        if hasattr(tokens, "tolist"):
            tokens = tokens.tolist()      # python ints once, not a numpy scalar per sequence
        for seq, tok in zip(step.seqs, tokens):
            st = seq.status
            if st is SeqStatus.FINISHED or st is SeqStatus.ABORTED:   # aborted while in flight
                seq.chunk = 0
                continue
            if seq.chunk:
                # a non-final chunk: its KV is cached, its sampled token is meaningless; the rest of
                # the prompt goes first in line for the next step
                seq.num_cached += seq.chunk
                seq.chunk = 0
                seq.status = SeqStatus.WAITING
                self.waiting.appendleft(seq)
                continue
            seq.num_cached = len(seq.prompt) + len(seq.output)
            if seq.append(tok, now) or seq.num_cached + 1 >= self.max_seq_len:
                if not seq.finished:
                    seq.finish("max_seq_len", now)
                self.bm.free_sequence(seq.seq_id)
                self.finished.append(seq)
                done.append(seq)
                continue
            p = seq.params
            self.native.admit(step.slot, seq.seq_id, seq.total_len, seq.output[-1],
                              p.max_new_tokens - len(seq.output), _eos_of(seq),
                              int(round(p.temperature * 1e4)) if p.temperature > 0 else 0, int(p.top_k),
                              int(round(p.top_p * 1e4)))
            self.live[seq.seq_id] = seq
        return done

    def pop_finished(self) -> List[Sequence]:
        f, self.finished = self.finished, []
        return f
