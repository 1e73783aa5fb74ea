"""Does the M = 256 decode gate|up scale with the CUs it occupies?  (stream-K feasibility probe)

gemm_wide runs the 8B gate|up (N = 28672, K = 4096) as 224 workgroups of 256 x 128 tiles: 32 of
the 256 CUs idle.  A stream-K form would give every CU 56 of the 64 K-tiles' worth of work.  This
times gemm_wide (SwiGLU epilogue) over N in {24576, 28672, 32768} (192 / 224 / 256 workgroups) and
over K in {3584, 4096} at N = 32768: if the 256-workgroup grid at K = 3584 runs in ~7/8 of the
224-workgroup K = 4096 grid, the kernel is bound per CU and stream-K would pay ~1/8 minus its
fix-up.  Weights rotate through > 512 MB of copies (cold, as in serving).  Median us.

    python bench/debug/wide_cu_scaling.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd.ops import gemm


def time_shape(m, n, k, rounds=7, calls=8):
    copies = max(2, int((512 << 20) // (n * k * 2)) + 1)
    ws = [torch.randn(n, k, device="cuda", dtype=torch.bfloat16) * 0.02 for _ in range(copies)]
    x = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    gemm.linear_wide(x, ws[0], swiglu=True)
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(calls):
            gemm.linear_wide(x, ws[i % copies], swiglu=True)
        e1.record()
        e1.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / calls)
    del ws
    return statistics.median(res)


def main():
    torch.manual_seed(0)
    for n, k in [(24576, 4096), (28672, 4096), (32768, 4096), (32768, 3584), (28672, 3584), (32768, 3072)]:
        t = time_shape(256, n, k)
        print(f"gate_up M=256 N={n:6d} K={k}  workgroups={n // 128:4d}  {t:7.1f} us  "
              f"({2 * 256 * n * k / t / 1e6:.0f} TF/s)", flush=True)


if __name__ == "__main__":
    main()
