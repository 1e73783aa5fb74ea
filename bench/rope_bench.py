"""RoPE + paged KV-append microbenchmark: is the decode-step cost the math or the cache scatter?

Same bytes, two slot patterns:
  decode  : T tokens, each appended to a DIFFERENT sequence's block (one 2-byte V^T column write
            per (head, dim) into a line no other token of the step touches)
  prefill : T tokens filling T/32 whole blocks (every V^T line fully written within the launch)
and a q-only baseline (kv heads = 0 cost is approximated by a tiny kv cache hit pattern).

    python bench/rope_bench.py [--tokens 256] [--iters 50]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd import knobs, ops
from distributed_llms_amd.ops import reference as ref


def timeit(fn, iters):
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
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    t, hq, hkv, d, bs = a.tokens, a.hq, a.hkv, a.d, 32
    dev = "cuda"
    nb = 8 * t + 64
    kc = torch.zeros(nb, hkv, bs, d, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros(nb, hkv, d, bs, dtype=torch.bfloat16, device=dev)
    qkv = torch.randn(t, (hq + 2 * hkv) * d, device=dev).to(torch.bfloat16)
    cs = ref.rope_cos_sin(d, 4096, 500000.0, None).to(dev)
    pos_dec = torch.full((t,), 161, dtype=torch.int32, device=dev)
    slots_dec = (torch.arange(t, device=dev, dtype=torch.int32) * 7 + 3) * bs + 1    # scattered blocks
    pos_pf = torch.arange(t, dtype=torch.int32, device=dev)
    slots_pf = torch.arange(t, dtype=torch.int32, device=dev) + 5 * bs               # whole blocks
    rows = []
    for name, pos, sl in (("decode", pos_dec, slots_dec), ("prefill", pos_pf, slots_pf)):
        f = lambda: ops.rope_cache_append(qkv, pos, cs, kc, vc, sl, hq, hkv, d)    # noqa: E731
        f()
        us = timeit(f, a.iters)
        moved = qkv.numel() * 2 + t * hq * d * 2 + 2 * t * hkv * d * 2
        rows.append(f"{name:8s} {us:8.2f} us  {moved / us / 1e6:6.2f} TB/s (bytes moved {moved / 1e6:.2f} MB)")
    # the engine's prefill form: K / V only (the attention kernel rotates q), V per token vs grouped
    for grouped in (False, True):
        with knobs.override(v_group_append=grouped):
            f = lambda: ops.rope_cache_append(qkv, pos_pf, cs, kc, vc, slots_pf, hq, hkv, d, write_q=False)  # noqa: E731
            f()
            us = timeit(f, a.iters)
        moved = 2 * t * hkv * d * 2 * 2      # read k, v; write k, v
        rows.append(f"prefill kv-only {'grouped V' if grouped else 'per-token V'}: {us:8.2f} us  "
                    f"{moved / us / 1e6:6.2f} TB/s (k/v bytes {moved / 1e6:.2f} MB)")
    print(f"tokens={t} hq={hq} hkv={hkv} d={d}")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
