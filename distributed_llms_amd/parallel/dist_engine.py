"""One process per GPU: bootstrap torch.distributed and build this rank's pipeline role.

World layout: ``world = dp * pp``; ranks ``[p*pp, (p+1)*pp)`` form pipeline ``p`` and
rank ``p*pp + s`` runs stage ``s``.  Backend "nccl" is RCCL on ROCm (activations over
xGMI); a gloo group carries the small CPU control messages (batch metadata, tokens).
"""
from __future__ import annotations

import datetime
import logging
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..config import EngineConfig
from ..engine.llm_engine import LLMEngine, build_stage, make_block_manager
from ..engine.runner import StageRunner, plan_kv_blocks
from .comm import DistTransport
from .pipeline import PipelineDriver, inflight_window, stage_worker_loop
from .planner import plan_units

log = logging.getLogger("dllm.dist")
# DLLM_PP_FINE=1: pipelines of dense models may cut at sub-layer units (planner.py).  Off by
# default: measured per-stage decode times on MI355X (profiles/pp_stage_balance.md) show the cuts'
# own costs (re-normalisation, half-width MLP GEMMs, wider hops) eat the balance they buy
FINE_UNITS = os.environ.get("DLLM_PP_FINE", "0") == "1"


@dataclass
class DistContext:
    """Rank layout: ``rank = (d * pp + s) * tp + t`` -- replica d, pipeline stage s, tensor-
    parallel rank t.  Lane (d, t) is the chain of the t-th TP ranks of replica d's stages: the
    activations and the sampled-ids ring of TP rank t travel along it (after a stage's
    all-reduce every TP rank holds the same hidden state, so each lane carries its own copy over
    its own xGMI links)."""
    rank: int
    world: int
    local_rank: int
    dp: int
    pp: int
    ctrl_group: object
    device: str
    data_group: object = None      # None = the default (RCCL) group
    ring_groups: tuple = ()        # per lane: the {stage 0, last stage} group of the ids ring closure
    tp: int = 1                    # tensor-parallel degree
    tpg: object = None             # this rank's TPGroup (parallel/tensor_parallel.py), None if tp == 1

    @property
    def host_staged(self) -> bool:
        return self.data_group is not None

    @property
    def replica(self) -> int:
        return self.rank // (self.pp * self.tp)

    @property
    def tp_rank(self) -> int:
        return self.rank % self.tp

    @property
    def pipeline_id(self) -> int:
        """Lane index (replica * tp + TP rank): one PipelineDriver per lane 0 of each replica."""
        return self.replica * self.tp + self.tp_rank

    @property
    def stage(self) -> int:
        return (self.rank // self.tp) % self.pp

    @property
    def pipeline_ranks(self):
        d, t = self.replica, self.tp_rank
        return [(d * self.pp + s) * self.tp + t for s in range(self.pp)]

    @property
    def ring_group(self):
        return self.ring_groups[self.pipeline_id] if self.ring_groups else None


def init_distributed(pp: Optional[int] = None, backend: Optional[str] = None,
                     timeout_s: float = 1800, tp: int = 1, moe: str = "tp") -> DistContext:
    """dp x pp x tp over the launched world (dp = world / (pp * tp); pp None = world / tp).
    ``moe``: how a TP group splits MoE experts ("tp": along I, "ep": whole experts per rank).

    Environment knobs (tests / rehearsal only):
      DLLM_SHARE_GPU=1       ranks share the visible GPUs round-robin (local_rank % device_count)
      DLLM_DATA_BACKEND=gloo activations go host-staged over a gloo group instead of RCCL -- the
                             cross-host TCP fallback, and the only way to run several GPU ranks on
                             one device (RCCL refuses: "Duplicate GPU detected")."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    dev_idx = local_rank
    if use_gpu and os.environ.get("DLLM_SHARE_GPU", "0") == "1":
        dev_idx = local_rank % max(1, torch.cuda.device_count())
    host_staged = use_gpu and os.environ.get("DLLM_DATA_BACKEND", "") == "gloo"
    if use_gpu:
        torch.cuda.set_device(dev_idx)
    backend = backend or ("gloo" if host_staged else "nccl" if use_gpu else "gloo")
    tmo = datetime.timedelta(seconds=timeout_s)
    if not dist.is_initialized():
        kw = dict(backend=backend, rank=rank, world_size=world, timeout=tmo)
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", dev_idx)
        dist.init_process_group(**kw)
    ctrl = dist.new_group(backend="gloo", timeout=tmo) if backend != "gloo" else dist.group.WORLD
    data = dist.new_group(backend="gloo", timeout=tmo) if host_staged else None
    tp = max(1, int(tp or 1))
    if world % tp:
        raise ValueError(f"world {world} not divisible by tp {tp}")
    pp = pp or world // tp
    if world % (pp * tp):
        raise ValueError(f"world {world} not divisible by pp {pp} x tp {tp}")
    dp = world // (pp * tp)
    p2p_backend = "gloo" if (host_staged or backend == "gloo") else "nccl"
    # new_group is collective: every rank creates every group, in the same order
    tpg = None
    if tp > 1:
        from .tensor_parallel import TPGroup
        for d in range(dp):
            for s in range(pp):
                ranks = [(d * pp + s) * tp + t for t in range(tp)]
                g = dist.new_group(ranks=ranks, backend=p2p_backend, timeout=tmo)
                c = dist.new_group(ranks=ranks, backend="gloo", timeout=tmo)
                if rank in ranks:
                    tpg = TPGroup(rank - ranks[0], tp, g, c, ranks[0], moe=moe)
    # one {first, last} group per lane for the sampled-ids ring closure
    rings = ()
    if pp > 1:
        rings = tuple(dist.new_group(ranks=[(d * pp) * tp + t, (d * pp + pp - 1) * tp + t], backend=p2p_backend,
                                     timeout=tmo)
                      for d in range(dp) for t in range(tp))
    return DistContext(rank, world, local_rank, dp, pp, ctrl, f"cuda:{dev_idx}" if use_gpu else "cpu", data,
                       rings, tp, tpg)


def resolve_transport(kind: str, device: str, host_staged: bool) -> str:
    """The activation transport a stage uses: CPU stages and host-staged GPU stages always ride
    torch.distributed (gloo) -- or HIP IPC when asked for (stages sharing one GPU); on GPUs "auto"
    is the native RCCL edge transport."""
    kind = os.environ.get("DLLM_TRANSPORT", "") or kind or "auto"    # env: test / rehearsal override
    if not str(device).startswith("cuda"):
        # CPU stages ride gloo -- except the RCCL transport's stand-in rehearsal (rccl_standin.py)
        from . import rccl_standin
        return "rccl" if kind == "rccl" and rccl_standin.enabled() else "torch"
    if host_staged:                     # stages sharing one GPU: HIP IPC if asked, else gloo
        from . import rccl_standin      # (or the RCCL transport over its stand-in: rehearsal)
        if kind == "rccl" and rccl_standin.enabled():
            return "rccl"
        return "ipc" if kind == "ipc" else "torch"
    return "rccl" if kind == "auto" else kind


def make_transport(ranks, stage: int, ctrl_group, data_group, device: str, ring_group=None, hop=None,
                   kind: str = "auto", timeout_s: float = 600.0):
    """Activation transport for one pipeline stage (see resolve_transport).  ``hop`` = (max rows,
    hidden, dtype, in-flight window) of an activation hop: every GPU transport sizes its static
    rings from it.  If the native RCCL communicators cannot be created on some rank, EVERY rank of
    the job falls back to torch.distributed's RCCL group (agreed over the control group), so a
    library or topology problem costs speed, not the run."""
    kind = resolve_transport(kind, device, data_group is not None)
    on_gpu = str(device).startswith("cuda")
    from . import rccl_standin
    if kind == "ipc" and on_gpu:
        from .ipc_transport import IpcTransport
        rows, hidden, dtype, window = hop
        return IpcTransport(ranks, stage, ctrl_group, device, rows, hidden, dtype, ring_group=ring_group,
                            window=window)
    if kind == "rccl" and (on_gpu or rccl_standin.enabled()):
        from .rccl_transport import RcclTransport
        rows, hidden, dtype, window = hop
        t, err = None, None
        try:
            t = RcclTransport(ranks, stage, ctrl_group, device, rows, hidden, dtype, ring_group=ring_group,
                              window=window, timeout_s=timeout_s)
        except Exception as e:          # noqa: BLE001 - reported, then the whole job agrees on a fallback
            err = e
        ok = torch.tensor([0 if err is None else 1], dtype=torch.int64)
        dist.all_reduce(ok, op=dist.ReduceOp.MAX, group=ctrl_group)
        if int(ok.item()) == 0:
            return t
        log.error("native RCCL transport unavailable (%s); every stage falls back to torch.distributed",
                  err if err is not None else "failed on another rank")
        if t is not None:
            t.abort()
    return DistTransport(ranks, stage, ctrl_group=ctrl_group, data_group=data_group, ring_group=ring_group,
                         hop=hop, device=device, timeout_s=timeout_s)


def agree_min(ctx: DistContext, value: int) -> int:
    t = torch.tensor([value], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=ctx.ctrl_group)
    return int(t.item())


def agree_max(ctx: DistContext, value: float) -> float:
    t = torch.tensor([value], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=ctx.ctrl_group)
    return float(t.item())


class RankRole:
    """What this rank runs: a full engine (pp == 1), a pipeline driver (stage 0, TP rank 0), a
    stage-0 TP peer of the driver, a pipeline follower, or a TP follower (pp == 1)."""

    def __init__(self, ctx: DistContext, ecfg: EngineConfig, hf_state=None):
        self.ctx = ctx
        self.ecfg = ecfg
        mcfg = ecfg.model_config()
        self.engine = None
        self.driver = None
        self.runner = None
        self.tp_follower = False        # dp x tp follower (pp == 1)
        self.lane_follower = False      # pp x tp: stage 0, TP rank > 0
        if ctx.tp > 1 and ctx.pp == 1:
            self._init_tp(ctx, ecfg, mcfg, hf_state)
            return
        self.plan = plan_units(mcfg, ctx.pp, batch=ecfg.max_batch, ctx=max(32, ecfg.max_seq_len // 2),
                               device=str(ctx.device), fine=FINE_UNITS and ctx.tp == 1)
        a, b = self.plan.ranges[ctx.stage]
        stage = build_stage(ecfg, a, b, device=ctx.device, shard_state=hf_state,
                            units=self.plan.unit_range(ctx.stage), tp=ctx.tpg, unit_group=self.plan.group)
        nb = plan_kv_blocks(mcfg, stage.num_layers, ecfg, stage.device, stage.hkv)
        nb = agree_min(ctx, nb)        # every stage of a pipeline must hold the same block ids
        if ctx.tp > 1:
            ecfg = ecfg.apply_overrides(use_graphs=False)      # collectives stay out of graph capture
        if ctx.pp == 1:
            ecfg1 = ecfg.apply_overrides(num_kv_blocks=nb)
            self.engine = LLMEngine(ecfg1, stage)
        else:
            self.runner = StageRunner(stage, ecfg, num_blocks=nb)
            # IPC slots fit the widest hop of the pipeline (a sub-layer cut adds the pending tensor)
            width = mcfg.hidden_size + (max(mcfg.qkv_size, mcfg.q_size, mcfg.hidden_size)
                                        if self.plan.group != 2 else 0)
            hop = (max(ecfg.max_prefill_tokens, ecfg.max_batch), width, stage.dtype,
                   inflight_window(ecfg, ctx.pp, stage.device))
            self.transport = make_transport(ctx.pipeline_ranks, ctx.stage, ctx.ctrl_group, ctx.data_group,
                                            ctx.device, ctx.ring_group, hop=hop, kind=ecfg.transport,
                                            timeout_s=ecfg.comm_timeout_s)
            if ctx.stage == 0 and ctx.tp_rank == 0:
                bm = make_block_manager(nb, ecfg.kv_block_size)
                self.driver = PipelineDriver(self.runner, self.transport, ecfg, bm)
            elif ctx.stage == 0:
                self.lane_follower = True
        log.info("rank %d: lane %d stage %d tp %d/%d layers [%d,%d) kv_blocks=%d", ctx.rank, ctx.pipeline_id,
                 ctx.stage, ctx.tp_rank, ctx.tp, a, b, nb)

    def _init_tp(self, ctx, ecfg, mcfg, hf_state):
        """dp x tp: every rank holds a TP shard of all layers; group rank 0 runs the engine."""
        from .planner import StagePlan
        stage = build_stage(ecfg, 0, mcfg.num_layers, device=ctx.device, shard_state=hf_state, tp=ctx.tpg)
        nb = plan_kv_blocks(mcfg, stage.num_layers, ecfg, stage.device, stage.hkv)
        nb = agree_min(ctx, nb)        # the leader's block ids index every rank's cache
        e = ecfg.apply_overrides(num_kv_blocks=nb, use_graphs=False)
        self.plan = StagePlan(((0, mcfg.num_layers),), (0.0,))
        if ctx.tpg.rank == 0:
            self.engine = LLMEngine(e, stage)
        else:
            self.runner = StageRunner(stage, e, num_blocks=nb)
            self.tp_follower = True
        log.info("rank %d: tp rank %d/%d of replica %d, kv_blocks=%d", ctx.rank, ctx.tpg.rank, ctx.tp,
                 ctx.rank // ctx.tp, nb)

    @property
    def is_driver(self) -> bool:
        return self.engine is not None or self.driver is not None

    def add_request(self, prompt, params):
        return (self.engine or self.driver).add_request(prompt, params)

    def run_round(self):
        """Drivers: run all queued requests to completion, then release followers.
        Followers: serve microbatches until the driver's ROUND_END."""
        if self.tp_follower:
            from .tensor_parallel import tp_follower_loop
            tp_follower_loop(self.runner, self.ctx.tpg, stop_on_round_end=True)
            return []
        if self.lane_follower:
            from .pipeline import stage0_tp_follower_loop
            stage0_tp_follower_loop(self.runner, self.transport, self.ctx.tpg, stop_on_round_end=True)
            return []
        if self.engine is not None:
            done = self.engine.run_until_done()
            self.engine.end_round()
            return done
        if self.driver is not None:
            done = self.driver.run_until_done()
            self.driver.end_round()
            return done
        stage_worker_loop(self.runner, self.transport, stop_on_round_end=True)
        return []

    def shutdown(self):
        if self.tp_follower:
            from .tensor_parallel import tp_follower_loop
            tp_follower_loop(self.runner, self.ctx.tpg, stop_on_round_end=False)
        elif self.lane_follower:
            from .pipeline import stage0_tp_follower_loop
            stage0_tp_follower_loop(self.runner, self.transport, self.ctx.tpg, stop_on_round_end=False)
        elif self.engine is not None:
            self.engine.shutdown()
        elif self.driver is not None:
            self.driver.shutdown()
        elif self.runner is not None:
            stage_worker_loop(self.runner, self.transport, stop_on_round_end=False)
        if hasattr(getattr(self, "transport", None), "close"):
            self.transport.close()          # IPC: unmap the peers' exports once this rank has drained
