"""Which Python call sites launch torch (at::native / rocclr) kernels inside a serving round?

    python bench/debug/torch_op_origins.py [--model llama3-8b] [--batch 256] [--rounds 1]

Runs one warmup round of bench.py's single-GPU engine, then profiles ``--rounds`` rounds with
torch.profiler (CUDA activities + Python stacks) and prints, for every kernel that is NOT one of
ours (``dllm::``), its count, total device time and the innermost package frames of the op that
launched it.  Graph-replayed kernels have no CPU op; they show up as '<graph replay>'.
"""
from __future__ import annotations

import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--rounds", type=int, default=1)
    a = ap.parse_args()
    import torch
    from torch.profiler import ProfilerActivity, profile
    from distributed_llms_amd.config import EngineConfig
    from distributed_llms_amd.engine.llm_engine import LLMEngine
    from distributed_llms_amd.engine.sequence import SamplingParams
    from bench import make_prompts

    eng = LLMEngine(EngineConfig(model=f"synthetic:{a.model}", max_batch=a.batch,
                                 max_prefill_tokens=max(16384, a.batch * a.prompt_len),
                                 max_seq_len=a.prompt_len + a.gen_len + 32))
    params = SamplingParams(max_new_tokens=a.gen_len, ignore_eos=True)
    vocab = eng.mcfg.vocab_size

    def round_(r):
        for p in make_prompts(a.batch, a.prompt_len, vocab, r):
            eng.add_request(p, params)
        eng.run_until_done()

    round_(10_000)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for r in range(a.rounds):
            round_(r)
        torch.cuda.synchronize()

    # kernel -> launching CPU op (by correlation through the event tree)
    evs = prof.events()
    by_kernel = collections.defaultdict(lambda: [0, 0.0, collections.Counter()])
    for e in evs:
        for k in getattr(e, "kernels", []) or []:
            name = k.name
            if name.startswith("dllm::") or "dllm" in name:
                continue
            stack = [f for f in (e.stack or []) if "distributed_llms_amd" in f or "bench" in f]
            site = " <- ".join(s.split("/")[-1] for s in stack[:4]) or e.name
            rec = by_kernel[name[:90]]
            rec[0] += 1
            rec[1] += k.duration / 1e3 if hasattr(k, "duration") else 0.0
            rec[2][f"{e.name} @ {site}"] += 1
    print(f"non-dllm kernels over {a.rounds} round(s):")
    for name, (n, ms, sites) in sorted(by_kernel.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:6d} {ms:9.2f} ms  {name}")
        for s, c in sites.most_common(4):
            print(f"            {c:5d}x {s}")
    print(prof.key_averages().table(sort_by="cuda_time_total", row_limit=25))


if __name__ == "__main__":
    main()
