"""Library GEMM time at a pipeline prefill microbatch (M = 8192 tokens, bench_dist.py), tuned table
vs hipBLASLt's default heuristic, Llama-3-8B / 70B projection shapes (us per call, warm):

    DLLM_TUNABLEOP_FILE=<csv> python bench/prefill_mb_gemm.py [--m 8192]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

SHAPES = {"qkv_8b": (6144, 4096), "o_8b": (4096, 4096), "gate_up_8b": (28672, 4096), "down_8b": (4096, 14336),
          "qkv_70b": (10240, 8192), "o_70b": (8192, 8192), "gate_up_70b": (57344, 8192), "down_70b": (8192, 28672)}


def t(fn, iters=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[8192])
    a = ap.parse_args()
    from distributed_llms_amd.ops.tuning import TUNED_CSV
    tun = torch.cuda.tunable
    for m in a.m:
        for name, (n, k) in SHAPES.items():
            x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
            w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
            tun.enable(False)
            heur = t(lambda: F.linear(x, w))
            tun.enable(True)
            tun.tuning_enable(False)
            tun.read_file(TUNED_CSV)
            tuned = t(lambda: F.linear(x, w))
            pf = 2.0 * m * n * k / 1e15
            print(f"{name:12s} M={m:6d} heuristic {heur:8.1f} us ({pf / heur * 1e6:.2f} PF)  tuned {tuned:8.1f} us "
                  f"({pf / tuned * 1e6:.2f} PF)", flush=True)
            del x, w
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
