"""Prefill attention microbenchmark: the kernel versions of csrc/kernels/attention.hip side by side.

    python bench/prefill_attn_bench.py [--versions 4 7 9]

Shapes: Llama-3 GQA (Hq 32, Hkv 8, D 128), whole prompts already in the paged cache (the
engine's prefill: rope_cache_append first, then attention over the sequence's own keys).
Reports us per call and the effective TFLOP/s of the causal QK^T + PV work.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd import knobs, ops
from distributed_llms_amd.ops import reference as ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--versions", nargs="+", default=["4", "7", "9"])
    ap.add_argument("--shapes", nargs="+", default=["256x128", "32x1024", "8x4096", "1x8192"],
                    help="BATCHxPROMPT_LEN")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rope", action="store_true",
                    help="the engine's form: q read from the raw qkv projection and rotated in the kernel")
    a = ap.parse_args()
    hq, hkv, d, bs = 32, 8, 128, 32
    print(f"{'shape':>10s} " + " ".join(f"{'v' + v + ' us':>10s} {'TF':>5s}" for v in a.versions))
    for sh in a.shapes:
        b, L = (int(t) for t in sh.split("x"))
        nblk = (L + bs - 1) // bs
        k = (torch.randn(b * nblk + 1, hkv, bs, d, device="cuda") * 0.5).to(torch.bfloat16)
        v = (torch.randn(b * nblk + 1, hkv, d, bs, device="cuda") * 0.5).to(torch.bfloat16)
        bt = (torch.arange(b * nblk, dtype=torch.int32, device="cuda") + 1).view(b, nblk)
        cu = torch.arange(0, (b + 1) * L, L, dtype=torch.int32, device="cuda")
        sl = torch.full((b,), L, dtype=torch.int32, device="cuda")
        q = torch.randn(b * L, hq, d, device="cuda").to(torch.bfloat16)
        qkv = torch.randn(b * L, (hq + 2 * hkv) * d, device="cuda").to(torch.bfloat16)
        pos = torch.arange(L, dtype=torch.int32, device="cuda").repeat(b)
        cs = ref.rope_cos_sin(d, L, 500000.0, device="cuda")
        flops = 4.0 * b * hq * d * L * (L + 1) / 2
        row = []
        for ver in a.versions:
            if a.rope:
                knobs.update({"prefill_attn": int(ver)})
            if a.rope:
                f = lambda: ops.paged_attention_prefill_rope(qkv, pos, cs, k, v, bt, cu, sl, hq, d, d ** -0.5,  # noqa: E731
                                                             max_q_len=L)
            else:
                f = lambda: ops.paged_attention_prefill(q, k, v, bt, cu, sl, d ** -0.5, version=int(ver))  # noqa: E731
            f()
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                e1.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            t = statistics.median(ts)
            row.append(f"{t:10.1f} {flops / t / 1e6:5.0f}")
        print(f"{sh:>10s} " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
