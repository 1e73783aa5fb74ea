#!/usr/bin/env python
"""Headline benchmark: output tokens/s (whole node) + p50 request latency, Llama-3-8B bf16.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...        (driver form for N > 1)

``python bench.py --gpus N`` (N > 1) with no launcher environment (WORLD_SIZE unset) launches
itself: the parent process touches no GPU API, starts N rank processes of this script (RANK /
LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT set, one process per GPU), passes
rank 0's JSON line through, and exits non-zero if any rank fails or the job outlives
``--launch-timeout``.

One *step* = one serving round: ``batch x N`` fresh requests (synthetic prompt ids of
``--prompt-len`` tokens) are submitted at once and the engine runs until every one of
them has produced ``--gen-len`` new tokens (prefill + continuous-batched decode, greedy,
EOS ignored).  W untimed rounds, then K timed rounds bracketed by a barrier +
torch.cuda.synchronize() on every rank; the max over ranks is reported.

  value       = K * batch * N * gen_len / elapsed      (output tokens/s, whole job)
  p50 latency = median request latency (submit -> last token) over the timed rounds

Parallelism: ``pp`` (default, BASELINE config 3: N workers each own a contiguous slice
of layers; activations hop stage->stage over RCCL/xGMI with N + 1 microbatches in flight),
``dp`` (N independent replicas) or ``tp`` (N-way tensor parallel groups, all-reduce per layer
half; ``--tp K`` = N/K replicas of K).  The microbatch size is fixed per GPU, so scaling is weak.
Weights are random-init (seeded, generated on device); prompts are synthetic ids.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "output tokens/sec (whole node) + p50 latency, Llama-3-8B across 1/2/4/8 workers"
BASELINE_VALUE = None   # reference publishes no number; comparator measured separately


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=256, help="sequences per GPU per round")
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--parallelism", choices=["pp", "dp", "tp"], default="pp")
    ap.add_argument("--tp", type=int, default=0,
                    help="tensor-parallel group size (--parallelism tp: default all ranks; with pp: "
                         "every pipeline stage is a TP group of this size, dp x pp x tp)")
    ap.add_argument("--moe", choices=["tp", "ep"], default="tp",
                    help="MoE models under TP: slice every expert along I (tp) or give each rank whole "
                         "experts (ep, expert parallelism)")
    ap.add_argument("--pp", type=int, default=0,
                    help="pipeline depth for --parallelism pp (default: all ranks); world/pp pipelines run as "
                         "data-parallel replicas, e.g. --gpus 8 --pp 4 = 2 pipelines of 4 stages")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--quant", choices=["none", "fp8"], default="none",
                    help="fp8: W8A8 e4m3 dense projections (opt-in serving mode; the headline stays bf16)")
    ap.add_argument("--streams", type=int, default=1, help="1-GPU engine: microbatch slots on separate streams")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--rate", type=float, default=0.0,
                    help="open-loop latency mode (1 GPU): requests arrive as a Poisson process of this many "
                         "requests/s (steps x batch requests in all) instead of a batch per round; reports "
                         "p50/p99 request latency, TTFT and ITL under that load (the headline mode is unchanged)")
    ap.add_argument("--comm-timeout", type=float, default=600.0,
                    help="pipeline ranks: a peer silent this long makes the rank raise (EngineConfig.comm_timeout_s)")
    ap.add_argument("--hang-dump", type=float, default=0.0,
                    help="diagnostics: dump every thread's Python stack every N seconds (0 = off)")
    ap.add_argument("--mixed-tokens", type=int, default=None,
                    help="EngineConfig.mixed_prefill_tokens: prompt tokens a step may add to running decode "
                         "rows (0 = prefill-first steps; default: the config's)")
    ap.add_argument("--launch-timeout", type=float, default=3600.0,
                    help="self-launched multi-GPU runs (--gpus N > 1 without torchrun): kill every rank and "
                         "exit non-zero after this many seconds")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--trace", default=None, metavar="DIR",
                    help="record a roctx/host/GPU timeline of the timed steps: DIR/trace_rank<r>.json "
                         "(Chrome format) and per-stage device busy %% in the JSON line")
    return ap.parse_args(argv)


def make_prompts(n, plen, vocab, seed):
    import numpy as np
    rng = np.random.default_rng(seed)
    return rng.integers(100, min(vocab, 30000), size=(n, plen)).tolist()


def _par_name(args, world):
    tp = args.tp or (world if args.parallelism == "tp" else 1)
    if args.parallelism == "pp":
        pp = args.pp or world // tp
    else:
        pp = 1
    dp = world // (pp * tp)
    ep = tp > 1 and getattr(args, "moe", "tp") == "ep" and "mixtral" in args.model
    parts = [f"dp{dp}" if dp > 1 else "", f"pp{pp}" if pp > 1 else "",
             (f"ep{tp}" if ep else f"tp{tp}") if tp > 1 else ""]
    name = "x".join(p for p in parts if p)
    return name or f"dp{world}"


def _knobs_changed():
    from distributed_llms_amd import knobs
    return knobs.changed()


def emit(args, world, elapsed, lat, extra, global_batch=None):
    """global_batch = requests per round over the whole job (default batch x world)."""
    global_batch = global_batch or args.batch * world
    tokens = args.steps * global_batch * args.gen_len
    value = tokens / elapsed
    rec = {
        "metric": METRIC, "value": round(value, 2), "unit": "tokens/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / args.steps, 3),
        "higher_is_better": True, "scaling": "weak",
        "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
        "dtype": "bf16" if args.quant == "none" else "fp8 (W8A8 projections, bf16 rest)",
        "data": "synthetic (random-init weights, random prompt ids)",
        "p50_latency_ms": round(1000 * statistics.median(lat), 3) if lat else None,
        # closed loop: every request of a round is submitted at once and the round ends when the
        # last one finishes, so a request's latency is its round's (prefill + gen_len steps)
        "latency_kind": "round (closed loop: all requests of a round submitted together)",
        "config": {"model": args.model, "global_batch": global_batch, "seq_len": args.prompt_len + args.gen_len,
                   "prompt_len": args.prompt_len, "gen_len": args.gen_len,
                   "parallelism": _par_name(args, world)},
        "kernel_knobs": _knobs_changed(),            # non-default kernel-dispatch knobs (none = defaults)
    }
    rec.update(extra)
    line = json.dumps(rec)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")


def start_trace(args):
    if not args.trace:
        return None
    from distributed_llms_amd.utils.tracing import get_tracer
    tr = get_tracer()
    tr.clear()
    return tr.enable(True)


def finish_trace(args, tr, elapsed, rank):
    """Export this rank's timeline; return its stage's device busy fraction over the timed steps."""
    tr.enable(False)
    os.makedirs(args.trace, exist_ok=True)
    util = tr.utilization(elapsed, cat="stage")
    tr.export_chrome(os.path.join(args.trace, f"trace_rank{rank}.json"), process_name=f"rank{rank}")
    return round(util["busy_frac"], 4)


def run_single(args):
    import torch
    from distributed_llms_amd.config import EngineConfig
    from distributed_llms_amd.engine.llm_engine import LLMEngine
    from distributed_llms_amd.engine.sequence import SamplingParams

    ecfg = EngineConfig(model=f"synthetic:{args.model}", max_batch=args.batch,
                        max_prefill_tokens=max(16384, args.batch * args.prompt_len),
                        max_seq_len=args.prompt_len + args.gen_len + 32, use_graphs=not args.no_graphs,
                        seed=args.seed, streams=args.streams, quant=args.quant)
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    t0 = time.perf_counter()
    eng = LLMEngine(ecfg)
    sync()
    load_s = time.perf_counter() - t0
    params = SamplingParams(max_new_tokens=args.gen_len, ignore_eos=True)
    vocab = eng.mcfg.vocab_size

    def round_(r):
        seqs = [eng.add_request(p, params) for p in make_prompts(args.batch, args.prompt_len, vocab, r)]
        eng.run_until_done()
        return seqs

    for r in range(args.warmup):
        round_(10_000 + r)
    sync()
    if eng.runner is not None:
        eng.runner.meter(True)
    tr = start_trace(args)
    lat, done = [], []
    t0 = time.perf_counter()
    for r in range(args.steps):
        seqs = round_(r)
        lat.extend(s.latency() for s in seqs)
        done.extend(seqs)
    sync()
    elapsed = time.perf_counter() - t0
    assert all(len(s.output) == args.gen_len for s in seqs)
    from distributed_llms_amd.utils.metrics import request_timing, seq_timing
    extra = {"load_s": round(load_s, 1), "transport": "none",
             "stage_busy_frac": [round(eng.runner.busy_seconds() / elapsed, 4) if eng.runner else None],
             **request_timing(*seq_timing(done))}
    if tr is not None:
        finish_trace(args, tr, elapsed, 0)
    emit(args, 1, elapsed, lat, extra)


def run_open_loop(args):
    """Latency under load (plan.md:470-473): one warmup round, then steps x batch requests whose
    arrivals are a Poisson process of ``--rate`` requests/s (seeded), admitted into the running
    engine as they arrive (continuous batching).  A request's latency counts from its scheduled
    arrival, so queueing behind a busy step is included.  One JSON line: p50 request latency is
    the value (lower is better); p99, TTFT, ITL, offered and achieved rates ride along."""
    import numpy as np
    import torch
    from distributed_llms_amd.config import EngineConfig
    from distributed_llms_amd.engine.llm_engine import LLMEngine
    from distributed_llms_amd.engine.sequence import SamplingParams
    from distributed_llms_amd.utils.metrics import percentile, request_timing, seq_timing

    ecfg = EngineConfig(model=f"synthetic:{args.model}", max_batch=args.batch,
                        max_prefill_tokens=max(16384, args.batch * args.prompt_len),
                        max_seq_len=args.prompt_len + args.gen_len + 32, use_graphs=not args.no_graphs,
                        seed=args.seed, streams=args.streams, quant=args.quant)
    if args.mixed_tokens is not None:
        ecfg = ecfg.apply_overrides(mixed_prefill_tokens=args.mixed_tokens)
    sync = torch.cuda.synchronize if torch.cuda.is_available() else (lambda: None)
    eng = LLMEngine(ecfg)
    params = SamplingParams(max_new_tokens=args.gen_len, ignore_eos=True)
    vocab = eng.mcfg.vocab_size
    for r in range(max(1, args.warmup)):
        for p in make_prompts(args.batch, args.prompt_len, vocab, 10_000 + r):
            eng.add_request(p, params)
        eng.run_until_done()
    sync()
    n = args.steps * args.batch
    rng = np.random.default_rng(args.seed + 7)
    arrivals = np.cumsum(rng.exponential(1.0 / args.rate, size=n))
    prompts = make_prompts(n, args.prompt_len, vocab, args.seed)
    seqs, i = [], 0
    t0 = time.perf_counter()
    while i < n or eng.has_work():
        now = time.perf_counter() - t0
        while i < n and arrivals[i] <= now:
            s = eng.add_request(prompts[i], params)
            s.arrival = t0 + float(arrivals[i])
            seqs.append(s)
            i += 1
        if eng.has_work():
            eng.step()
        elif i < n:
            time.sleep(max(0.0, float(arrivals[i]) - (time.perf_counter() - t0)))
    sync()
    elapsed = time.perf_counter() - t0
    assert all(len(s.output) == args.gen_len for s in seqs)
    lat = [s.latency() for s in seqs]
    rec = {"metric": f"request latency under Poisson load (open loop), {args.model}", "value":
           round(1000 * percentile(lat, 50), 3), "unit": "ms", "higher_is_better": False, "n_gpus": 1,
           "requests": n, "offered_rate_rps": args.rate, "achieved_rate_rps": round(n / elapsed, 3),
           "p50_latency_ms": round(1000 * percentile(lat, 50), 3),
           "p99_latency_ms": round(1000 * percentile(lat, 99), 3),
           "latency_kind": "request (open loop: scheduled arrival -> last token)",
           "output_tok_per_s": round(n * args.gen_len / elapsed, 2), "dtype": "bf16" if args.quant == "none" else "fp8",
           "data": "synthetic (random-init weights, random prompt ids)",
           "config": {"model": args.model, "max_batch": args.batch, "prompt_len": args.prompt_len,
                      "gen_len": args.gen_len, "mixed_prefill_tokens": ecfg.mixed_prefill_tokens},
           "mixed_steps": eng.scheduler.num_mixed, "kernel_knobs": _knobs_changed(),
           **request_timing(*seq_timing(seqs))}
    line = json.dumps(rec)
    print(line, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(line + "\n")


def _free_port() -> int:
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(args, argv) -> int:
    """``--gpus N`` without a launcher: start N rank processes of this script (subprocess, never
    exec; this process imports nothing that initialises HIP), rank r on GPU r.  Rank 0's stdout
    (the JSON line) passes through; the other ranks' stdout goes to stderr.  The first rank to fail
    ends the job: the others are terminated and its exit code is returned; so is 124 when the job
    outlives ``--launch-timeout``."""
    import signal
    import subprocess
    n = args.gpus
    port = _free_port()
    cmd = [sys.executable, os.path.abspath(__file__)] + list(sys.argv[1:] if argv is None else argv)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr))

    def stop_all(sig=signal.SIGTERM):
        for p in procs:
            if p.poll() is None:
                try:
                    p.send_signal(sig)
                except OSError:
                    pass

    def on_signal(signum, _frame):
        stop_all()
        raise SystemExit(128 + signum)

    old = {sg: signal.signal(sg, on_signal) for sg in (signal.SIGTERM, signal.SIGINT)}
    t_end = time.monotonic() + args.launch_timeout if args.launch_timeout > 0 else None
    rc = 0
    clean = False
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0]
                print(f"bench.py: a rank exited with {rc}; stopping the others", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                clean = True
                break
            if t_end is not None and time.monotonic() > t_end:
                rc = 124
                print(f"bench.py: ranks still running after --launch-timeout {args.launch_timeout:.0f} s",
                      file=sys.stderr, flush=True)
                break
            time.sleep(0.2)
    finally:
        if not clean:
            stop_all()
            deadline = time.monotonic() + 20
            while time.monotonic() < deadline and any(p.poll() is None for p in procs):
                time.sleep(0.2)
            stop_all(signal.SIGKILL)
        for p in procs:
            p.wait()
        for sg, h in old.items():
            signal.signal(sg, h)
    return rc


def main(argv=None):
    args = parse(argv)
    if args.hang_dump > 0:
        # every rank prints all its threads' Python stacks every hang_dump seconds (stderr): where a
        # stuck pipeline's host is waiting
        import faulthandler
        faulthandler.dump_traceback_later(args.hang_dump, repeat=True)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.rate > 0:
        if world > 1 or args.gpus > 1:
            raise SystemExit("--rate (open-loop latency mode) runs on one GPU")
        return run_open_loop(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        rc = launch_ranks(args, argv)
        if rc:
            raise SystemExit(rc)
        return None
    if world > 1 or args.gpus > 1:
        from distributed_llms_amd.parallel.bench_dist import run_distributed
        return run_distributed(args, emit, make_prompts, start_trace, finish_trace)
    run_single(args)


if __name__ == "__main__":
    main()
