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
from ..utils.tracing import get_tracer
from .comm import STOP, Transport

log = logging.getLogger("dllm.pipeline")

ROUND_END = -2     # control marker: followers return to their caller (bench round barrier)
FLUSH = -3         # control marker: the last stage must hand back the tokens it still holds
_MARKERS = (STOP, ROUND_END, FLUSH)


def _marker(code: int) -> np.ndarray:
    return np.array([code], dtype=np.int32)


class _TokenReturn:
    """Last stage: sampled ids go D2H asynchronously; a microbatch's tokens are sent only after
    the NEXT microbatch has been launched, so the GPU never idles on the host's sync + send."""

    def __init__(self, transport: Transport, max_rows: int, device):
        self.t = transport
        self.cuda = torch.device(device).type == "cuda"
        self.bufs = [torch.empty(max_rows, dtype=torch.int32).pin_memory() if self.cuda else None for _ in range(2)]
        self.events = [torch.cuda.Event() if self.cuda else None for _ in range(2)]
        self.i = 0
        self.pending = None

    def push(self, step_id: int, ids: torch.Tensor):
        n = ids.shape[0]
        if self.cuda:
            if n > self.bufs[self.i].shape[0]:
                self.bufs[self.i] = torch.empty(n, dtype=torch.int32).pin_memory()
            self.bufs[self.i][:n].copy_(ids, non_blocking=True)
            self.events[self.i].record()
            item = (step_id, n, self.i)
            self.i ^= 1
        else:
            item = (step_id, n, ids.numpy().astype(np.int32))
        self.flush()
        self.pending = item

    def flush(self):
        if self.pending is None:
            return
        step_id, n, ref = self.pending
        self.pending = None
        if self.cuda:
            self.events[ref].synchronize()
            ids = self.bufs[ref][:n].numpy()
        else:
            ids = ref
        self.t.send_tokens(np.concatenate([np.array([step_id, n], np.int32), ids.astype(np.int32)]))


def stage_worker_loop(runner: StageRunner, transport: Transport, stop_on_round_end: bool = True) -> str:
    """Run a non-first stage until STOP (returns "stop") or ROUND_END (returns "round")."""
    st = runner.stage
    h = st.cfg.hidden_size
    last = transport.stage == transport.num_stages - 1
    ret = _TokenReturn(transport, runner.ecfg.max_batch, st.device) if last else None
    tr = get_tracer()
    while True:
        arr = transport.recv_meta()
        if arr.shape[0] == 1 and arr[0] in _MARKERS:
            if last:
                ret.flush()
            else:
                transport.send_meta(arr) if arr[0] != STOP else transport.send_stop()
            if arr[0] == STOP:
                return "stop"
            if arr[0] == ROUND_END and stop_on_round_end:
                return "round"
            continue
        hb = HostBatch.unpack(arr)
        if not last:
            transport.send_meta(arr)          # let the next stage post its receive early
        with tr.span("pp.recv_hidden", cat="comm", step=hb.step_id):
            hidden = transport.recv_hidden(hb.num_tokens, h, st.dtype, st.device)
        out = runner.execute(hb, hidden)
        if last:
            ret.push(hb.step_id, sample(out, **hb.sampling_args()))
        else:
            with tr.span("pp.send_hidden", cat="comm", step=hb.step_id):
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
        # one microbatch per stage keeps every stage busy only if the ring closure (last stage ->
        # tokens -> stage 0 scheduling) were free; one spare slot hides that turnaround
        self.num_slots = num_slots or (ecfg.microbatches if ecfg.microbatches > 0 else transport.num_stages + 1)
        self.scheduler = Scheduler(block_manager, self.num_slots, ecfg.max_batch, ecfg.max_prefill_tokens,
                                   ecfg.max_seq_len)
        self.mcfg = runner.stage.cfg
        self.inflight: Deque[Tuple[Step, int]] = collections.deque()
        self.busy = [False] * self.num_slots
        self.step_id = 0
        self.num_steps = 0
        self.stall_s = 0.0
        self._flushed = True

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
        self._flushed = False
        out = self.runner.execute(hb)
        self.t.send_hidden(out)
        self.inflight.append((step, self.step_id))
        self.busy[slot] = True
        self.step_id += 1
        self.num_steps += 1
        return True

    def _complete_oldest(self) -> List[Sequence]:
        if len(self.inflight) == 1 and not self._flushed:
            # the last stage holds the newest step's tokens until the next microbatch arrives;
            # waiting on that step with nothing else to send would deadlock without a flush
            self.t.send_meta(_marker(FLUSH))
            self._flushed = True
        step, sid = self.inflight.popleft()
        t0 = time.perf_counter()
        with get_tracer().span("pp.wait_tokens", cat="comm", step=sid):
            arr = self.t.recv_tokens()
        self.stall_s += time.perf_counter() - t0
        if int(arr[0]) != sid or int(arr[1]) != step.size:
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
    from .planner import plan_units

    mcfg = ecfg.model_config()
    plan = plan_units(mcfg, num_stages, batch=ecfg.max_batch, ctx=max(32, ecfg.max_seq_len // 2))
    hub = LoopbackHub(num_stages)
    runners = []
    for s, (a, b) in enumerate(plan.ranges):
        stage = build_stage(ecfg, a, b, device=device, shard_state=hf_state, units=plan.unit_range(s))
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
