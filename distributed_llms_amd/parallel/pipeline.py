"""Layer-sharded pipeline execution with microbatch overlap (BASELINE config 3/4/5).

The reference broadcasts every request to every worker and never moves activations
between them (``src/master/node.py:256-269``).  Here a pipeline of
``pp`` stages owns contiguous layer slices; stage 0 (:class:`PipelineDriver`) runs the
continuous-batching scheduler with ``num_slots`` (>= pp) microbatch slots and issues one
microbatch after another, so every stage has work in flight:

    stage 0:  schedule(slot) -> meta -> stage-0 forward -> send hidden      (no wait)
    stage s:  recv meta -> recv hidden -> forward -> send hidden / sample
    last:     logits -> sample -> tokens back to stage 0 (ring closure)

Stage 0 only blocks on a slot's sampled tokens when it is that slot's turn again, which
is ``num_slots`` microbatches later -- by then the tokens have normally arrived.
"""
from __future__ import annotations

import collections
import logging
import time
from typing import Deque, List, Optional, Tuple

import numpy as np
import torch

from ..config import EngineConfig
from ..engine.batch import HostBatch, build_host_batch
from ..engine.runner import StageRunner
from ..engine.sampler import sample
from ..engine.scheduler import Scheduler, Step
from ..engine.sequence import SamplingParams, Sequence
from .comm import STOP, Transport

log = logging.getLogger("dllm.pipeline")

ROUND_END = -2     # control marker: followers return to their caller (bench round barrier)


def _marker(code: int) -> np.ndarray:
    return np.array([code], dtype=np.int32)


def stage_worker_loop(runner: StageRunner, transport: Transport, stop_on_round_end: bool = True) -> str:
    """Run a non-first stage until STOP (returns "stop") or ROUND_END (returns "round")."""
    st = runner.stage
    h = st.cfg.hidden_size
    last = transport.stage == transport.num_stages - 1
    while True:
        arr = transport.recv_meta()
        if arr.shape[0] == 1 and arr[0] in (STOP, ROUND_END):
            if not last:
                transport.send_meta(arr) if arr[0] == ROUND_END else transport.send_stop()
            if arr[0] == STOP:
                return "stop"
            if stop_on_round_end:
                return "round"
            continue
        hb = HostBatch.unpack(arr)
        if not last:
            transport.send_meta(arr)          # let the next stage post its receive early
        hidden = transport.recv_hidden(hb.num_tokens, h, st.dtype, st.device)
        out = runner.execute(hb, hidden)
        if last:
            ids = sample(out, **hb.sampling_args())
            ids = ids.cpu().numpy().astype(np.int32)
            transport.send_tokens(np.concatenate([np.array([hb.step_id, ids.shape[0]], np.int32), ids]))
        else:
            transport.send_hidden(out)


class PipelineDriver:
    """Stage 0: scheduler + block manager owner; issues microbatches into the pipeline."""

    def __init__(self, runner: StageRunner, transport: Transport, ecfg: EngineConfig, block_manager,
                 num_slots: Optional[int] = None):
        assert transport.stage == 0 and transport.num_stages >= 2
        self.runner = runner
        self.t = transport
        self.ecfg = ecfg
        self.bm = block_manager
        self.num_slots = num_slots or max(ecfg.microbatches, transport.num_stages)
        self.scheduler = Scheduler(block_manager, self.num_slots, ecfg.max_batch, ecfg.max_prefill_tokens,
                                   ecfg.max_seq_len)
        self.mcfg = runner.stage.cfg
        self.inflight: Deque[Tuple[Step, int]] = collections.deque()
        self.busy = [False] * self.num_slots
        self.step_id = 0
        self.num_steps = 0
        self.stall_s = 0.0

    def add_request(self, prompt: List[int], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None) -> Sequence:
        seq = Sequence(list(prompt), params or SamplingParams(), eos_token_id=self.mcfg.eos_token_id,
                       request_id=request_id)
        self.scheduler.add(seq)
        return seq

    def _issue(self, slot: int) -> bool:
        step = self.scheduler.schedule(slot)
        if step is None:
            return False
        hb = build_host_batch(step, self.bm, self.ecfg.kv_block_size,
                              None if step.is_prefill else self.runner.max_blocks, self.step_id)
        self.t.send_meta(hb.pack())
        out = self.runner.execute(hb)
        self.t.send_hidden(out)
        self.inflight.append((step, self.step_id))
        self.busy[slot] = True
        self.step_id += 1
        self.num_steps += 1
        return True

    def _complete_oldest(self) -> List[Sequence]:
        step, sid = self.inflight.popleft()
        t0 = time.perf_counter()
        arr = self.t.recv_tokens()
        self.stall_s += time.perf_counter() - t0
        if int(arr[0]) != sid or int(arr[1]) != len(step.seqs):
            raise RuntimeError(f"pipeline out of order: got step {arr[0]} n={arr[1]}, expected {sid}")
        done = self.scheduler.complete(step, arr[2:2 + int(arr[1])], time.perf_counter())
        self.busy[step.slot] = False
        return done

    def poll(self) -> List[Sequence]:
        """One pass over all slots; returns finished sequences."""
        issued = False
        for slot in range(self.num_slots):
            while self.busy[slot]:
                self._complete_oldest()
            if self._issue(slot):
                issued = True
        if not issued and self.inflight:
            self._complete_oldest()
        return self.scheduler.pop_finished()

    def has_work(self) -> bool:
        return self.scheduler.has_work() or bool(self.inflight)

    def run_until_done(self) -> List[Sequence]:
        done = []
        while self.has_work():
            done.extend(self.poll())
        done.extend(self.scheduler.pop_finished())
        return done

    def end_round(self):
        self.t.send_meta(_marker(ROUND_END))

    def shutdown(self):
        self.t.send_stop()
        if hasattr(self.t, "drain"):
            self.t.drain()

    def generate(self, prompts, params: Optional[SamplingParams] = None) -> List[List[int]]:
        seqs = [self.add_request(p, params) for p in prompts]
        self.run_until_done()
        return [s.output for s in seqs]


def run_loopback_pipeline(ecfg: EngineConfig, num_stages: int, prompts, params: SamplingParams,
                          device: Optional[str] = None, hf_state=None):
    """N stage threads in ONE process sharing one device (1-GPU pipeline emulation / tests)."""
    import threading

    from ..engine.llm_engine import build_stage, make_block_manager
    from .comm import LoopbackHub
    from .planner import plan_stages

    mcfg = ecfg.model_config()
    plan = plan_stages(mcfg, num_stages)
    hub = LoopbackHub(num_stages)
    runners = []
    for s, (a, b) in enumerate(plan.ranges):
        stage = build_stage(ecfg, a, b, device=device, shard_state=hf_state)
        runners.append(StageRunner(stage, ecfg, num_blocks=ecfg.num_kv_blocks or 512))
    errors = []
    # capture every stage's decode graphs up front, one at a time: concurrent captures from
    # several threads of one process are not something to rely on
    for r in runners:
        r.warmup_graphs(ctx_buckets=(min(256, ecfg.max_seq_len),))

    def follower(s):
        try:
            dev = runners[s].stage.device
            if dev.type == "cuda":
                with torch.cuda.stream(torch.cuda.Stream(dev)):
                    stage_worker_loop(runners[s], hub.transport(s), stop_on_round_end=False)
            else:
                stage_worker_loop(runners[s], hub.transport(s), stop_on_round_end=False)
        except BaseException as e:  # pragma: no cover - surfaced below
            errors.append(e)
            hub.tokens.put(np.array([-99, 0], np.int32))

    threads = [threading.Thread(target=follower, args=(s,), daemon=True) for s in range(1, num_stages)]
    for th in threads:
        th.start()
    bm = make_block_manager(runners[0].num_blocks, ecfg.kv_block_size)
    drv = PipelineDriver(runners[0], hub.transport(0), ecfg, bm)
    try:
        outs = drv.generate(prompts, params)
    except RuntimeError as e:
        if errors:
            raise errors[0] from e
        raise
    finally:
        drv.shutdown()
        for th in threads:
            th.join(timeout=60)
    if errors:
        raise errors[0]
    return outs, drv, plan
