"""Layer-sharded pipeline execution with microbatch overlap (BASELINE config 3/4/5).

The reference broadcasts every request to every worker and never moves activations
between them (``src/master/node.py:256-269``).  Here a pipeline of
``pp`` stages owns contiguous layer slices; stage 0 (:class:`PipelineDriver`) runs the
continuous-batching scheduler with ``num_slots`` (>= pp) microbatch slots and issues one
microbatch after another, so every stage has work in flight:

    stage 0:  schedule(slot) -> meta -> stage-0 forward -> send hidden -> post ids receive
    stage s:  recv meta -> recv hidden -> forward -> send hidden
    last:     ... -> logits -> sample -> send ids to stage 0 (ring closure, device to device)

A slot's next decode step is issued with LOOKAHEAD: its rows and metadata come from the native
batcher (positions advanced past the step still in flight) and its input ids are the in-flight
step's sampled ids, received on the device and gathered there.  The host reads those ids one
step later, for bookkeeping only, so neither the host nor the control plane is on the ring's
critical path: a slot's round trip is the stages' GPU time plus the hops, against ``num_slots``
microbatches of stage-0 work.  Steps that need the host first (prefill admission, preemption,
sampled sequences' stop checks after a prefill) fall back to completing the slot's step before
scheduling (knobs.pp_lookahead off: always).
"""
from __future__ import annotations

import collections
import logging
import os
import time
from typing import Deque, List, Optional

import numpy as np
import torch

from .. import knobs
from ..config import EngineConfig, pipeline_slots, resolve_device  # noqa: F401  (pipeline_slots re-exported)
from ..engine.batch import HostBatch, build_host_batch
from ..engine.runner import StageRunner
from ..engine.sampler import sample
from ..engine.scheduler import Scheduler, Step
from ..engine.sequence import SamplingParams, Sequence
from ..utils.tracing import get_tracer
from .comm import STOP, PendingIds, Transport

log = logging.getLogger("dllm.pipeline")

ROUND_END = -2     # control marker: followers return to their caller (bench round barrier)
_MARKERS = (STOP, ROUND_END)


def _marker(code: int) -> np.ndarray:
    return np.array([code], dtype=np.int32)


def stage_worker_loop(runner: StageRunner, transport: Transport, stop_on_round_end: bool = True) -> str:
    """Run a non-first stage until STOP (returns "stop") or ROUND_END (returns "round")."""
    st = runner.stage
    h = st.in_width
    last = transport.stage == transport.num_stages - 1
    tr = get_tracer()
    while True:
        arr = transport.recv_meta()
        if arr.shape[0] == 1 and arr[0] in _MARKERS:
            if not last:
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
            # the ids go out as soon as they are sampled; the send is stream-ordered behind them
            if st.tp.enabled:       # vocab-parallel head: every TP rank derives the same ids
                from .tensor_parallel import tp_sample
                transport.send_ids(tp_sample(out, st.tp, hb.sampling_args()))
            else:
                transport.send_ids(sample(out, **hb.sampling_args()))
        else:
            with tr.span("pp.send_hidden", cat="comm", step=hb.step_id):
                transport.send_hidden(out)


class _Issued:
    """A microbatch stage 0 has issued and not yet completed on the host."""
    __slots__ = ("step", "sid", "ids")

    def __init__(self, step: Step, sid: int, ids: PendingIds):
        self.step, self.sid, self.ids = step, sid, ids


def inflight_window(ecfg: EngineConfig, pp: int, device=None) -> int:
    """Most microbatches the driver ever has in flight: two per slot (a step and its lookahead
    successor).  Microbatch n is issued only after n - window completed at stage 0, i.e. after
    every stage finished it -- transports with slot rings deeper than this never need credits."""
    return 2 * pipeline_slots(ecfg, pp, device)


class PipelineDriver:
    """Stage 0: scheduler + block manager owner; issues microbatches into the pipeline."""

    def __init__(self, runner: StageRunner, transport: Transport, ecfg: EngineConfig, block_manager,
                 num_slots: Optional[int] = None):
        assert transport.stage == 0 and transport.num_stages >= 2
        self.runner = runner
        self.t = transport
        self.ecfg = ecfg
        self.bm = block_manager
        self.num_slots = num_slots or pipeline_slots(ecfg, transport.num_stages, runner.stage.device)
        self.scheduler = Scheduler(block_manager, self.num_slots, ecfg.max_batch, ecfg.max_prefill_tokens,
                                   ecfg.max_seq_len, ecfg.mixed_prefill_tokens)
        self.mcfg = runner.stage.cfg
        self.device = runner.stage.device
        self.inflight: Deque[_Issued] = collections.deque()           # issue order
        self.per_slot: List[Deque[_Issued]] = [collections.deque() for _ in range(self.num_slots)]
        self.lookahead = knobs.K.pp_lookahead
        # pp x tp: the stage-0 TP peers replay every issue on their own lanes
        self.tp = runner.stage.tp if runner.stage.tp.enabled else None
        self.step_id = 0
        self.num_steps = 0
        self.num_lookahead = 0
        self.stall_s = 0.0

    def add_request(self, prompt: List[int], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None) -> Sequence:
        seq = Sequence(list(prompt), params or SamplingParams(), eos_token_id=self.mcfg.eos_token_id,
                       request_id=request_id)
        self.scheduler.add(seq)
        return seq

    def _issue(self, step: Step, ids_dev: Optional[torch.Tensor] = None):
        assert len(self.inflight) < 2 * self.num_slots, "in-flight window exceeded (see inflight_window)"
        hb = build_host_batch(step, self.bm, self.ecfg.kv_block_size,
                              None if step.is_prefill else self.runner.max_blocks, self.step_id)
        if self.tp is not None:
            self.tp.bcast_meta(_tp_issue_msg(hb.pack(), ids_dev is not None, step.keep))
        self.t.send_meta(hb.pack())
        out = self.runner.execute(hb, ids_dev=ids_dev) if ids_dev is not None else self.runner.execute(hb)
        self.t.send_hidden(out)
        # the ids receive is posted right away: receives are matched in issue order
        it = _Issued(step, self.step_id, self.t.recv_ids(step.size, self.device))
        self.inflight.append(it)
        self.per_slot[step.slot].append(it)
        self.step_id += 1
        self.num_steps += 1

    def _complete_oldest(self) -> List[Sequence]:
        it = self.inflight.popleft()
        q = self.per_slot[it.step.slot]
        assert q[0] is it
        q.popleft()
        t0 = time.perf_counter()
        with get_tracer().span("pp.wait_tokens", cat="comm", step=it.sid):
            toks = it.ids.host()
        self.stall_s += time.perf_counter() - t0
        if toks.shape[0] != it.step.size:
            raise RuntimeError(f"pipeline out of order: step {it.sid} got {toks.shape[0]} ids for {it.step.size} rows")
        return self.scheduler.complete(it.step, toks, time.perf_counter())

    def _issue_lookahead(self, slot: int) -> bool:
        """The slot's next decode step on the device ids of its in-flight step (see module doc)."""
        if not self.lookahead or self.scheduler.waiting:
            return False
        q = self.per_slot[slot]
        if len(q) != 1 or q[0].step.is_prefill:
            return False
        step = self.scheduler.schedule_lookahead(slot)
        if step is None:
            return False
        prev = q[0].ids.wait()                   # stream-ordered behind the ids' arrival
        if step.keep is not None:
            keep = torch.from_numpy(np.asarray(step.keep, dtype=np.int64))
            prev = prev.index_select(0, keep.to(prev.device, non_blocking=True) if prev.is_cuda else keep)
        self._issue(step, ids_dev=prev)
        self.num_lookahead += 1
        return True

    def poll(self) -> List[Sequence]:
        """One pass over all slots; returns finished sequences."""
        issued = False
        for slot in range(self.num_slots):
            if self.per_slot[slot] and self._issue_lookahead(slot):
                issued = True
                # at most two steps of a slot in flight: absorb the older one (its ids are needed
                # on the host only now, one full cycle after they were sampled)
                self._complete_oldest()
                continue
            while self.per_slot[slot]:
                self._complete_oldest()
            step = self.scheduler.schedule(slot)
            if step is not None:
                self._issue(step)
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
        if self.tp is not None:
            self.tp.bcast_meta(_marker(ROUND_END))
        self.t.send_meta(_marker(ROUND_END))

    def shutdown(self):
        if self.tp is not None:
            self.tp.bcast_meta(_marker(STOP))
        self.t.send_stop()
        if hasattr(self.t, "drain"):
            self.t.drain()

    def generate(self, prompts, params=None) -> List[List[int]]:
        """``params``: one SamplingParams for all prompts, or a list (one per prompt)."""
        plist = params if isinstance(params, (list, tuple)) else [params] * len(prompts)
        seqs = [self.add_request(p, q) for p, q in zip(prompts, plist)]
        self.run_until_done()
        return [s.output for s in seqs]


def _tp_issue_msg(packed: np.ndarray, lookahead: bool, keep) -> np.ndarray:
    """[kind, n_keep, keep..., packed HostBatch...]: kind 1 = ids in the batch, 2 = lookahead on
    the device ids of the slot's previous step (n_keep -1: every row)."""
    keep = np.asarray(keep, dtype=np.int32) if keep is not None else np.zeros(0, np.int32)
    head = np.array([2 if lookahead else 1, keep.shape[0] if keep.shape[0] else -1], np.int32)
    return np.concatenate([head, keep, packed])


def stage0_tp_follower_loop(runner: StageRunner, transport: Transport, tp, stop_on_round_end: bool = True) -> str:
    """pp x tp, stage 0, TP rank > 0: replay each microbatch the driver (TP rank 0 of the same
    stage) issues -- same metadata, same lookahead -- on this rank's own lane: its own activation
    hop to the next stage's TP rank, its own ids ring from the last stage's TP rank."""
    newest = {}                                   # slot -> PendingIds of its newest step
    while True:
        msg = tp.bcast_meta(None)
        if msg.shape[0] == 1 and int(msg[0]) in _MARKERS:
            if int(msg[0]) == STOP:
                transport.send_stop()
                if hasattr(transport, "drain"):
                    transport.drain()
                return "stop"
            transport.send_meta(msg.copy())
            if stop_on_round_end:
                return "round"
            continue
        kind, n_keep = int(msg[0]), int(msg[1])
        keep = msg[2:2 + max(n_keep, 0)].astype(np.int64)
        packed = msg[2 + max(n_keep, 0):].copy()
        hb = HostBatch.unpack(packed)
        transport.send_meta(packed)
        if kind == 2:
            prev = newest[hb.slot].wait()
            if n_keep >= 0:
                k = torch.from_numpy(keep)
                prev = prev.index_select(0, k.to(prev.device) if prev.is_cuda else k)
            out = runner.execute(hb, ids_dev=prev)
        else:
            out = runner.execute(hb)
        transport.send_hidden(out)
        old = newest.get(hb.slot)
        newest[hb.slot] = transport.recv_ids(hb.num_seqs, runner.stage.device)
        if old is not None and not runner.stage.device.type == "cuda":
            old.wait()                           # CPU (gloo): let the receive complete before dropping it


def run_loopback_pipeline(ecfg: EngineConfig, num_stages: int, prompts, params: SamplingParams,
                          device: Optional[str] = None, hf_state=None):
    """N stage threads in ONE process sharing one device (1-GPU pipeline emulation / tests)."""
    import threading

    from ..engine.llm_engine import build_stage, make_block_manager
    from .comm import LoopbackHub
    from .planner import plan_units

    mcfg = ecfg.model_config()
    plan = plan_units(mcfg, num_stages, batch=ecfg.max_batch, ctx=max(32, ecfg.max_seq_len // 2),
                      device=str(device or resolve_device(ecfg.device)),
                      fine=os.environ.get("DLLM_PP_FINE", "0") == "1")
    hub = LoopbackHub(num_stages)
    runners = []
    for s, (a, b) in enumerate(plan.ranges):
        stage = build_stage(ecfg, a, b, device=device, shard_state=hf_state, units=plan.unit_range(s),
                            unit_group=plan.group)
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
            hub.ids.put((RuntimeError(f"stage {s} failed"), None))

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
