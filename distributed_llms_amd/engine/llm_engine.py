"""Single-process engine: one worker owning all layers (BASELINE config 2), also the
building block for data-parallel replicas.

Loop: ``schedule -> host batch -> stage forward (eager prefill / graph-replayed decode)
-> sample -> complete``.  The pipeline engine (parallel/pipeline.py) runs the same
scheduler and stage executor split across processes.
"""
from __future__ import annotations

import collections
import logging
import time
from typing import Iterable, List, Optional

import numpy as np
import torch

from .. import _ext, knobs
from ..config import EngineConfig, resolve_device, torch_dtype
from ..models.stage import ModelStage
from .batch import build_host_batch
from .graphs import SCRATCH_SEQ_ID
from .runner import StageRunner
from .sampler import sample
from .scheduler import Scheduler, Step
from .sequence import SamplingParams, Sequence

log = logging.getLogger("dllm.engine")


def make_block_manager(num_blocks: int, block_size: int):
    bm = _ext.runtime().BlockManager(num_blocks, block_size)
    # block 0 is the scratch block padded decode rows write into
    assert bm.ensure_capacity(SCRATCH_SEQ_ID, 1)
    assert bm.block_table(SCRATCH_SEQ_ID) == [0]
    return bm


def build_stage(ecfg: EngineConfig, layer_start: int = 0, layer_end: Optional[int] = None,
                device: Optional[str] = None, shard_state=None, units=None, tp=None,
                unit_group: int = 2) -> ModelStage:
    """``units`` / ``unit_group``: the stage's unit range (parallel/planner.py StagePlan)."""
    mcfg = ecfg.model_config()
    layer_end = mcfg.num_layers if layer_end is None else layer_end
    dev = resolve_device(device or ecfg.device)
    dtype = torch_dtype(ecfg.dtype)
    stage = ModelStage(mcfg, layer_start, layer_end, device=dev, dtype=dtype, units=units, tp=tp,
                       unit_group=unit_group)
    if shard_state is not None:
        stage.load_hf_state(shard_state)
    else:
        stage.init_synthetic(ecfg.seed)
    return stage.quantize(ecfg.quant)


class LLMEngine:
    def __init__(self, ecfg: EngineConfig, stage: Optional[ModelStage] = None):
        ecfg.validate() if ecfg.shard_dir is None else None
        self.ecfg = ecfg
        self.stage = stage or build_stage(ecfg)
        if not (self.stage.is_first and self.stage.is_last):
            raise ValueError("LLMEngine needs a stage owning every layer")
        self.mcfg = self.stage.cfg
        gpu = self.stage.device.type == "cuda"
        # tensor parallel leader: every step's metadata goes to the group before it runs, and the
        # followers join its collectives (parallel/tensor_parallel.py); synchronous steps, one
        # slot, eager launches (collectives stay out of graph capture)
        self.tp = self.stage.tp if self.stage.tp.enabled else None
        if self.tp is not None:
            ecfg = self.ecfg = ecfg.apply_overrides(use_graphs=False, streams=1)
        self.num_slots = max(1, ecfg.streams) if gpu else 1
        self.runner = StageRunner(self.stage, ecfg, num_slots=self.num_slots)
        self.bm = make_block_manager(self.runner.num_blocks, ecfg.kv_block_size)
        # max_batch is the engine's total decode batch, split evenly over the slots
        per_slot = -(-ecfg.max_batch // self.num_slots)
        self.scheduler = Scheduler(self.bm, self.num_slots, per_slot, ecfg.max_prefill_tokens, ecfg.max_seq_len,
                                   ecfg.mixed_prefill_tokens)
        self.step_id = 0
        self.num_prefill_tokens = 0
        self.num_decode_tokens = 0
        # async slots: each has its own stream, pinned token buffer and completion event
        self.inflight = collections.deque()
        self.busy = [False] * self.num_slots
        # lookahead: issue a slot's next decode step before completing the one in flight (input
        # ids gathered on device from the in-flight step's samples), so the host's complete /
        # schedule / build work overlaps the GPU instead of idling it (knobs.lookahead off: synchronous)
        self.lookahead = gpu and knobs.K.lookahead and self.tp is None
        self.num_lookahead = 0
        if gpu:
            dev = self.stage.device
            self.streams = [torch.cuda.Stream(dev) for _ in range(self.num_slots)]
            # two pinned token buffers + events per slot: with lookahead two steps of a slot are in flight
            self.tok_host = [[torch.empty(max(ecfg.max_batch, 1), dtype=torch.int32).pin_memory() for _ in range(2)]
                             for _ in range(self.num_slots)]
            self.events = [[torch.cuda.Event() for _ in range(2)] for _ in range(self.num_slots)]
            self.tok_i = [0] * self.num_slots

    # ------------------------------------------------------------ requests
    def add_request(self, prompt: List[int], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None) -> Sequence:
        seq = Sequence(list(prompt), params or SamplingParams(), eos_token_id=self.mcfg.eos_token_id,
                       request_id=request_id)
        self.scheduler.add(seq)
        return seq

    def has_work(self) -> bool:
        return self.scheduler.has_work() or bool(self.inflight)

    # ------------------------------------------------------------ stepping
    def _host_batch(self, step: Step):
        hb = build_host_batch(step, self.bm, self.ecfg.kv_block_size,
                              None if step.is_prefill else self.runner.max_blocks, self.step_id)
        if self.tp is not None:
            self.tp.bcast_meta(hb.pack())
        self.step_id += 1
        if step.is_prefill:
            self.num_prefill_tokens += hb.num_tokens
        else:
            self.num_decode_tokens += hb.num_tokens
        return hb

    def execute_step(self, step: Step) -> List[int]:
        """Synchronous execution of one step (CPU path / tests)."""
        hb = self._host_batch(step)
        logits = self.runner.execute(hb, slot=step.slot)
        ids = self._sample(logits, hb)
        return ids.cpu().tolist()

    def _sample(self, logits, hb):
        if self.tp is not None:
            from ..parallel.tensor_parallel import tp_sample
            return tp_sample(logits, self.tp, hb.sampling_args())
        return sample(logits, **hb.sampling_args())

    def _launch(self, step: Step, hb, slot: int, ids_src: Optional[torch.Tensor] = None, keep=None):
        """``ids_src`` (lookahead): the in-flight step's sampled ids on the device, rows ``keep``
        (None = all) become this step's input ids.  The gather runs on the slot's stream, behind
        the sampling that produces ``ids_src``."""
        s = self.streams[slot]
        s.wait_stream(torch.cuda.current_stream())
        i = self.tok_i[slot]
        self.tok_i[slot] ^= 1
        with torch.cuda.stream(s):
            ids_dev = None
            if ids_src is not None:
                ids_dev = ids_src if keep is None else ids_src.index_select(
                    0, torch.from_numpy(np.asarray(keep, dtype=np.int64)).pin_memory().to(ids_src.device,
                                                                                          non_blocking=True))
            logits = self.runner.execute(hb, slot=slot, ids_dev=ids_dev)
            ids = self._sample(logits, hb)
            n = ids.shape[0]
            self.tok_host[slot][i][:n].copy_(ids, non_blocking=True)
            self.events[slot][i].record(s)
        self.inflight.append((step, slot, n, i, ids))
        self.busy[slot] = True

    def _issue(self, slot: int) -> bool:
        step = self.scheduler.schedule(slot)
        if step is None:
            return False
        self._launch(step, self._host_batch(step), slot)
        return True

    def _issue_lookahead(self, slot: int) -> bool:
        """Issue the decode step that follows the slot's newest in-flight decode step, before that
        step's tokens reach the host.  Sequences that step will finish by length are left out;
        one finishing by EOS (unknowable here) computes one throw-away row, skipped by complete().
        Safe for the KV pool: blocks freed on completion are only reused by later steps on the
        same stream.  Returns False (caller falls back to the synchronous path) when anything
        needs the host first: waiting requests, non-decode steps, KV growth failures."""
        if not self.lookahead or self.scheduler.waiting or not self.inflight:
            return False
        prev, pslot, pn, _, pids = self.inflight[-1]
        if pslot != slot or prev.is_prefill or len(self.inflight) > 1:
            return False
        step = self.scheduler.schedule_lookahead(slot)      # native: rows, packed metadata, keep
        if step is None:
            return False
        hb = self._host_batch(step)
        self._launch(step, hb, slot, ids_src=pids[:pn], keep=step.keep)
        self.num_lookahead += 1
        return True

    def _complete_oldest(self):
        step, slot, n, i, _ = self.inflight.popleft()
        self.events[slot][i].synchronize()
        self.scheduler.complete(step, self.tok_host[slot][i][:n].numpy(), time.perf_counter())
        self.busy[slot] = any(e[1] == slot for e in self.inflight)

    def step(self) -> List[Sequence]:
        """One pass over the microbatch slots; returns sequences that finished."""
        if self.stage.device.type != "cuda":
            st = self.scheduler.schedule(0)
            if st is not None:
                toks = self.execute_step(st)
                self.scheduler.complete(st, toks, time.perf_counter())
            return self.scheduler.pop_finished()
        issued = False
        for slot in range(self.num_slots):
            if self.busy[slot] and self._issue_lookahead(slot):
                # the step after the in-flight one is queued behind it: now absorb the older one
                self._complete_oldest()
                issued = True
                continue
            while self.busy[slot]:
                self._complete_oldest()
            if self._issue(slot):
                issued = True
        if not issued and self.inflight:
            self._complete_oldest()
        return self.scheduler.pop_finished()

    def run_until_done(self) -> List[Sequence]:
        done = []
        while self.has_work():
            done.extend(self.step())
        done.extend(self.scheduler.pop_finished())
        return done

    def end_round(self):
        """Tensor-parallel leader: release the followers' step loops (bench round barrier)."""
        if self.tp is not None:
            from ..parallel.tensor_parallel import ROUND_END
            self.tp.bcast_meta(np.array([ROUND_END], np.int32))

    def shutdown(self):
        if self.tp is not None:
            from ..parallel.tensor_parallel import STOP
            self.tp.bcast_meta(np.array([STOP], np.int32))

    def generate(self, prompts: Iterable[List[int]], params=None) -> List[List[int]]:
        """``params``: one SamplingParams for all prompts, or a list (one per prompt)."""
        prompts = list(prompts)
        plist = params if isinstance(params, (list, tuple)) else [params] * len(prompts)
        seqs = [self.add_request(p, q) for p, q in zip(prompts, plist)]
        self.run_until_done()
        return [s.output for s in seqs]
