"""Per-stage decode time of a pipeline plan, measured one stage at a time on one GPU.

An N-GPU pipeline runs at the pace of its slowest stage.  This builds every stage of
``plan_units(cfg, pp, fine=...)`` in turn (synthetic weights on the device, its paged KV pool),
replays its decode graph for a batch-``B`` microbatch at context ``--ctx`` and reports the stage
times and max / mean -- the balance the planner's cost model predicts, measured on MI355X:

    python bench/pp_stage_times.py [--model llama3-8b] [--pp 2 4 8] [--batch 256] [--ctx 144]
"""
import argparse
import gc
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.batch import build_host_batch
from distributed_llms_amd.engine.llm_engine import build_stage, make_block_manager
from distributed_llms_amd.engine.runner import StageRunner
from distributed_llms_amd.engine.scheduler import Scheduler
from distributed_llms_amd.engine.sequence import SamplingParams, Sequence
from distributed_llms_amd.parallel.planner import plan_units


def decode_batch(ecfg, batch, ctx, nb, vocab=32000):
    """A decode HostBatch of ``batch`` sequences whose context reaches ``ctx`` (bookkeeping only:
    the prefill is scheduled and completed on the host, its KV left as allocated).  The decode
    step's input ids are random: with one shared id every sequence's first-stage activations are
    identical, and an MoE router sends the whole batch to the same two experts -- the first stage
    of Mixtral then streamed a quarter of the expert weights of the others and timed 0.57x."""
    bm = make_block_manager(nb, ecfg.kv_block_size)
    sch = Scheduler(bm, 1, batch, batch * ctx, ecfg.max_seq_len)
    for _ in range(batch):
        sch.add(Sequence([7] * (ctx - 1), SamplingParams(max_new_tokens=64, ignore_eos=True)))
    step = sch.schedule(0)
    assert step.is_prefill and step.size == batch
    sch.complete(step, np.random.default_rng(0).integers(3, vocab, batch).astype(np.int32), 0.0)
    step = sch.schedule(0)
    assert not step.is_prefill
    return build_host_batch(step, bm, ecfg.kv_block_size, -(-ecfg.max_seq_len // ecfg.kv_block_size), 1)


def time_stage(ecfg, plan, s, hb, nb, iters, device):
    a, b = plan.ranges[s]
    st = build_stage(ecfg, a, b, device=device, units=plan.unit_range(s), unit_group=plan.group)
    runner = StageRunner(st, ecfg, num_blocks=nb)
    hidden = None if st.is_first else (torch.randn(hb.num_tokens, st.in_width, device=device) * 0.1).to(st.dtype)
    gpu = device != "cpu"
    sync = torch.cuda.synchronize if gpu else (lambda: None)
    for _ in range(3):
        runner.execute(hb, hidden)
    sync()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        for _ in range(10):
            runner.execute(hb, hidden)
        sync()
        ts.append((time.perf_counter() - t0) * 1e5)     # us per replay
    del runner, st, hidden
    gc.collect()
    if gpu:
        torch.cuda.empty_cache()
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--pp", type=int, nargs="+", default=[2, 4, 8])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--ctx", type=int, default=144)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--device", default="cuda")
    a = ap.parse_args()
    ecfg = EngineConfig(model=f"synthetic:{a.model}", max_batch=a.batch, max_seq_len=a.ctx + 64,
                        graph_batch_sizes=(a.batch,), device=a.device,
                        dtype="bfloat16" if a.device != "cpu" else "float32")
    cfg = ecfg.model_config()
    nb = a.batch * -(-(a.ctx + 64) // ecfg.kv_block_size) + 2
    hb = decode_batch(ecfg, a.batch, a.ctx, nb, vocab=get_model_config(a.model).vocab_size)
    for pp in a.pp:
        for fine in (False, True):
            plan = plan_units(cfg, pp, batch=a.batch, ctx=a.ctx, device="cuda", fine=fine)
            us = [time_stage(ecfg, plan, s, hb, nb, a.iters, a.device) for s in range(pp)]
            mean = sum(us) / pp
            print(f"pp{pp} {'sub-layer' if plan.group == 5 else 'half-layer':10s} units {list(plan.units)}\n"
                  f"    stage us {[round(u, 1) for u in us]}  max/mean {max(us) / mean:.4f} "
                  f"(model {plan.imbalance():.4f})  slowest {max(us):.1f} us", flush=True)


if __name__ == "__main__":
    main()
