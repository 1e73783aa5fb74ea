"""Multi-rank body of bench.py (torchrun, one process per GPU)."""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist

from ..config import EngineConfig
from ..engine.sequence import SamplingParams
from ..utils.metrics import request_timing, seq_timing
from .dist_engine import RankRole, agree_max, init_distributed


def _sync(ctx):
    if torch.cuda.is_available() and ctx.device != "cpu":
        torch.cuda.synchronize()
    dist.barrier(group=ctx.ctrl_group)


def run_distributed(args, emit, make_prompts, start_trace=None, finish_trace=None):
    pp = (getattr(args, "pp", 0) or None) if args.parallelism == "pp" else 1
    tp = getattr(args, "tp", 0) or (int(os.environ.get("WORLD_SIZE", "1")) if args.parallelism == "tp" else 1)
    ctx = init_distributed(pp=pp, tp=tp, moe=getattr(args, "moe", "tp"), timeout_s=600)
    world = ctx.world
    # pipeline: prefill in ~8K-token microbatches (M large enough for full-rate GEMMs) so the
    # fill/drain bubble of the prefill phase is (pp-1) x ~8K-token stage times, not (pp-1) x a
    # whole slot's prompts (256 x 128 = 32K tokens per microbatch would idle ~15 % of a round at pp8)
    pf_tokens = max(16384, args.batch * args.prompt_len) if ctx.pp == 1 else max(8192, args.prompt_len)
    # tensor parallel: synchronous eager steps (collectives stay out of graph capture)
    ecfg = EngineConfig(model=f"synthetic:{args.model}", max_batch=args.batch,
                        max_prefill_tokens=pf_tokens,
                        max_seq_len=args.prompt_len + args.gen_len + 32,
                        use_graphs=not args.no_graphs and ctx.tp == 1,
                        num_workers=ctx.pp, seed=args.seed, quant=getattr(args, "quant", "none"),
                        comm_timeout_s=getattr(args, "comm_timeout", 600.0))
    t0 = time.perf_counter()
    role = RankRole(ctx, ecfg)
    _sync(ctx)
    load_s = time.perf_counter() - t0
    params = SamplingParams(max_new_tokens=args.gen_len, ignore_eos=True)
    vocab = ecfg.model_config().vocab_size
    # requests per pipeline per round: `batch` per microbatch slot (pp=1: the engine's batch)
    slots = role.driver.num_slots if role.driver is not None else 1
    slots = int(agree_max(ctx, slots))
    per_pipe = args.batch * slots

    def one_round(r):
        seqs = []
        if role.is_driver:
            prompts = make_prompts(per_pipe, args.prompt_len, vocab, r * 1000 + ctx.pipeline_id)
            seqs = [role.add_request(p, params) for p in prompts]
        role.run_round()
        return seqs

    for r in range(args.warmup):
        one_round(10_000 + r)
    _sync(ctx)
    runner = role.runner if role.runner is not None else getattr(role.engine, "runner", None)
    if runner is not None:
        runner.meter(True)
    tr = start_trace(args) if start_trace else None
    tp_ = getattr(role, "transport", None)
    hop0 = tp_.hop_stats() if tp_ is not None else {}
    lat, done = [], []
    t0 = time.perf_counter()
    for r in range(args.steps):
        seqs = one_round(r)
        lat.extend(s.latency() for s in seqs)
        done.extend(seqs)
    _sync(ctx)
    elapsed = agree_max(ctx, time.perf_counter() - t0)
    hop1 = tp_.hop_stats() if tp_ is not None else {}
    if role.is_driver:
        assert all(len(s.output) == args.gen_len for s in seqs), "incomplete generations"
    # gather latencies to rank 0
    obj = [None] * world
    dist.all_gather_object(obj, (lat, seq_timing(done)), group=ctx.ctrl_group)
    all_lat = [x for part in obj for x in part[0]]
    all_ttft = [x for part in obj for x in part[1][0]]
    all_itl = [x for part in obj for x in part[1][1]]
    if tr is not None:
        finish_trace(args, tr, elapsed, ctx.rank)
    # per-rank device busy fraction over the timed rounds, and what the data plane ran on
    mine = {"busy": round(runner.busy_seconds() / elapsed, 4) if runner is not None else None}
    mine["transport"] = getattr(tp_, "kind", "none") if tp_ is not None else "none"
    from . import rccl_standin
    if mine["transport"] == "rccl" and rccl_standin.enabled():
        mine["transport"] = "rccl-standin"          # the result was NOT measured over RCCL
    d = {k: hop1.get(k, 0) - hop0.get(k, 0) for k in hop1}
    mine["hop_tx"] = (d.get("hidden_tx", 0) + d.get("ids_tx", 0)) / elapsed   # device-plane bytes / s out
    mine["hop_rx"] = (d.get("hidden_rx", 0) + d.get("ids_rx", 0)) / elapsed
    mine["meta"] = (d.get("meta_tx", 0) + d.get("meta_rx", 0)) / elapsed
    mine["rccl_comm_ranks"] = list(getattr(tp_, "comm_ranks", []) or [])
    info = [None] * world
    dist.all_gather_object(info, mine, group=ctx.ctrl_group)
    busy = [i["busy"] for i in info]
    if ctx.rank == 0:
        pj = role.plan.to_json()
        extra = {"load_s": round(load_s, 1), "stage_ranges": pj["ranges"], "backend": dist.get_backend()}
        if "units" in pj:
            extra["stage_units"] = {"group": pj["group"], "ranges": pj["units"]}
        if role.driver is not None:
            extra["driver_stall_s"] = round(role.driver.stall_s, 3)
        extra["microbatch_slots"] = slots
        extra["stage_busy_frac"] = busy
        kinds = sorted({i["transport"] for i in info})
        extra["transport"] = kinds[0] if len(kinds) == 1 else kinds
        # a pipeline run names the RCCL data plane only when every rank sat on an RCCL edge:
        # otherwise the field says how many did (never a bare "rccl" over a partial plane)
        n_rccl = sum(1 for i in info if i["rccl_comm_ranks"])
        if ctx.pp > 1 and extra["transport"] in ("rccl", "rccl-standin") and n_rccl != world:
            extra["transport"] = f"{extra['transport']} on {n_rccl} of {world} ranks"
        # every native RCCL communicator appears on both of its ranks: count them once.  The
        # pipeline data plane is built from 2-rank EDGE communicators (stage s <-> s + 1, plus
        # the ids ring closure last -> first), so rccl_comm_nranks is [2] at any N -- the number
        # of edges (rccl_comms) and of ranks on them (rccl_ranks) is what grows with N
        extra["rccl_comms"] = sum(len(i["rccl_comm_ranks"]) for i in info) // 2
        extra["rccl_ranks"] = sum(1 for i in info if i["rccl_comm_ranks"])
        extra["rccl_comm_nranks"] = sorted({n for i in info for n in i["rccl_comm_ranks"]})
        # per-rank activation / ids traffic over the timed rounds (xGMI hops), MB/s
        extra["hop_tx_MBps"] = [round(i["hop_tx"] / 1e6, 3) for i in info]
        extra["hop_rx_MBps"] = [round(i["hop_rx"] / 1e6, 3) for i in info]
        extra["meta_MBps"] = [round(i["meta"] / 1e6, 3) for i in info]
        extra.update(request_timing(all_ttft, all_itl))
        emit(args, world, elapsed, all_lat, extra, global_batch=per_pipe * ctx.dp)
    role.shutdown()
    _sync(ctx)
    dist.destroy_process_group()
