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

import torch

from .. import _ext
from ..config import EngineConfig, resolve_device, torch_dtype
from ..models.stage import ModelStage
from .batch import build_host_batch
from .graphs import SCRATCH_SEQ_ID
from .runner import StageRunner
from .sampler import sample, step_sampling_args
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
                device: Optional[str] = None, shard_state=None, units=None) -> ModelStage:
    mcfg = ecfg.model_config()
    layer_end = mcfg.num_layers if layer_end is None else layer_end
    dev = resolve_device(device or ecfg.device)
    dtype = torch_dtype(ecfg.dtype)
    stage = ModelStage(mcfg, layer_start, layer_end, device=dev, dtype=dtype, units=units)
    if shard_state is not None:
        stage.load_hf_state(shard_state)
    else:
        stage.init_synthetic(ecfg.seed)
    return stage


class LLMEngine:
    def __init__(self, ecfg: EngineConfig, stage: Optional[ModelStage] = None):
        ecfg.validate() if ecfg.shard_dir is None else None
        self.ecfg = ecfg
        self.stage = stage or build_stage(ecfg)
        if not (self.stage.is_first and self.stage.is_last):
            raise ValueError("LLMEngine needs a stage owning every layer")
        self.mcfg = self.stage.cfg
        gpu = self.stage.device.type == "cuda"
        self.num_slots = max(1, ecfg.streams) if gpu else 1
        self.runner = StageRunner(self.stage, ecfg, num_slots=self.num_slots)
        self.bm = make_block_manager(self.runner.num_blocks, ecfg.kv_block_size)
        # max_batch is the engine's total decode batch, split evenly over the slots
        per_slot = -(-ecfg.max_batch // self.num_slots)
        self.scheduler = Scheduler(self.bm, self.num_slots, per_slot, ecfg.max_prefill_tokens, ecfg.max_seq_len)
        self.step_id = 0
        self.num_prefill_tokens = 0
        self.num_decode_tokens = 0
        # async slots: each has its own stream, pinned token buffer and completion event
        self.inflight = collections.deque()
        self.busy = [False] * self.num_slots
        if gpu:
            dev = self.stage.device
            self.streams = [torch.cuda.Stream(dev) for _ in range(self.num_slots)]
            self.tok_host = [torch.empty(max(ecfg.max_batch, 1), dtype=torch.int32).pin_memory()
                             for _ in range(self.num_slots)]
            self.events = [torch.cuda.Event() for _ in range(self.num_slots)]

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
        ids = sample(logits, **step_sampling_args(step.seqs))
        return ids.cpu().tolist()

    def _issue(self, slot: int) -> bool:
        step = self.scheduler.schedule(slot)
        if step is None:
            return False
        hb = self._host_batch(step)
        s = self.streams[slot]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            logits = self.runner.execute(hb, slot=slot)
            ids = sample(logits, **step_sampling_args(step.seqs))
            n = ids.shape[0]
            self.tok_host[slot][:n].copy_(ids, non_blocking=True)
            self.events[slot].record(s)
        self.inflight.append((step, slot, n))
        self.busy[slot] = True
        return True

    def _complete_oldest(self):
        step, slot, n = self.inflight.popleft()
        self.events[slot].synchronize()
        self.scheduler.complete(step, self.tok_host[slot][:n].tolist(), time.perf_counter())
        self.busy[slot] = False

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

    def generate(self, prompts: Iterable[List[int]], params: Optional[SamplingParams] = None) -> List[List[int]]:
        seqs = [self.add_request(p, params) for p in prompts]
        self.run_until_done()
        return [s.output for s in seqs]
