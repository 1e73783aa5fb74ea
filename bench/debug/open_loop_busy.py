"""How busy is the GPU under open-loop load?  (mixed prefill + decode steps run eagerly, and the
engine only issues a decode step ahead -- lookahead -- when nothing is waiting.)

    python bench/debug/open_loop_busy.py [--rate 176] [--mixed 8192] [--seconds 4]

Runs bench.py's open-loop engine (Llama-3-8B, prompt 128 / gen 128, Poisson arrivals) for a
warm-up, then profiles a steady-state window with torch.profiler: device kernel time vs wall
time, and the step mix (mixed / prefill / decode, lookahead or not) with the mean wall time of
each kind of engine.step() call.
"""
import argparse
import collections
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=176.0)
    ap.add_argument("--mixed", type=int, default=8192)
    ap.add_argument("--seconds", type=float, default=4.0)
    a = ap.parse_args()
    import numpy as np
    import torch
    from torch.profiler import ProfilerActivity, profile
    from distributed_llms_amd.config import EngineConfig
    from distributed_llms_amd.engine.llm_engine import LLMEngine
    from distributed_llms_amd.engine.sequence import SamplingParams
    from bench import make_prompts

    eng = LLMEngine(EngineConfig(model="synthetic:llama3-8b", max_batch=256, max_prefill_tokens=32768,
                                 max_seq_len=128 + 128 + 32, mixed_prefill_tokens=a.mixed))
    params = SamplingParams(max_new_tokens=128, ignore_eos=True)
    vocab = eng.mcfg.vocab_size
    for p in make_prompts(256, 128, vocab, 10_000):
        eng.add_request(p, params)
    eng.run_until_done()
    torch.cuda.synchronize()
    n = int(a.rate * (a.seconds + 8))
    rng = np.random.default_rng(7)
    arrivals = np.cumsum(rng.exponential(1.0 / a.rate, size=n))
    prompts = make_prompts(n, 128, vocab, 0)
    kinds = collections.Counter()
    wall = collections.defaultdict(float)
    i, t0 = 0, time.perf_counter()
    prof, started, t_start = None, False, 0.0
    while i < n or eng.has_work():
        now = time.perf_counter() - t0
        while i < n and arrivals[i] <= now:
            eng.add_request(prompts[i], params)
            i += 1
        if not started and now > 4.0:                 # steady state: profile a window
            prof = profile(activities=[ProfilerActivity.CUDA])
            prof.__enter__()
            started, t_start = True, time.perf_counter()
        if started and prof is not None and time.perf_counter() - t_start > a.seconds:
            torch.cuda.synchronize()
            w = time.perf_counter() - t_start
            prof.__exit__(None, None, None)
            busy = sum(e.self_device_time_total for e in prof.key_averages()) / 1e6
            print(f"rate {a.rate} mixed {a.mixed}: window {w:.2f} s, device kernel time {busy:.2f} s "
                  f"({100 * busy / w:.1f} % busy)")
            print("steps in window:", dict(kinds), {k: round(1e3 * v / max(1, kinds[k]), 2) for k, v in wall.items()},
                  "(mean ms per engine.step() call)")
            prof = None
            break
        if eng.has_work():
            la = eng.num_lookahead
            mixed = eng.scheduler.num_mixed
            s0 = time.perf_counter()
            eng.step()
            dt = time.perf_counter() - s0
            if started:
                k = "mixed" if eng.scheduler.num_mixed > mixed else ("lookahead" if eng.num_lookahead > la else "other")
                kinds[k] += 1
                wall[k] += dt
        else:
            time.sleep(max(0.0, float(arrivals[i]) - (time.perf_counter() - t0)))


if __name__ == "__main__":
    main()
