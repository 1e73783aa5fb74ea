"""Paged decode attention microbenchmark (Llama-3 GQA shapes) on one MI355X.

Times N back-to-back launches between two events (the GPU never idles, so host launch
overhead is excluded) and reports us/call and KV bytes streamed per second, sweeping the
split-plan target (``ops.DECODE_TARGET_WAVES``).

    python bench/attn_bench.py [--batch 64 256] [--ctx 192 1024 4096]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import distributed_llms_amd.ops as ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[16, 64, 256])
    ap.add_argument("--ctx", type=int, nargs="+", default=[192, 1024, 4096])
    ap.add_argument("--targets", type=int, nargs="+", default=[512, 1024, 2048, 4096])
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev, bs = "cuda", 32
    print(f"{'B':>4s} {'ctx':>5s} " + " ".join(f"{'t' + str(t):>16s}" for t in a.targets))
    for b in a.batch:
        for ctx in a.ctx:
            mb = -(-ctx // bs) + 1
            nb = b * mb + 1
            kc = torch.randn(nb, a.hkv, bs, a.d, device=dev).to(torch.bfloat16)
            vc = torch.randn(nb, a.hkv, a.d, bs, device=dev).to(torch.bfloat16)
            perm = torch.randperm(nb - 1, device=dev)[: b * mb].to(torch.int32) + 1      # scattered blocks
            bt = perm.view(b, mb).contiguous()
            sl = torch.full((b,), ctx, dtype=torch.int32, device=dev)
            q = torch.randn(b, a.hq, a.d, device=dev).to(torch.bfloat16)
            kv_bytes = b * ctx * a.hkv * a.d * 2 * 2
            cells = []
            for t in a.targets:
                ops.DECODE_TARGET_WAVES = t
                f = lambda: ops.paged_attention_decode(q, kc, vc, bt, sl, 0.088, max_ctx=ctx)   # noqa: E731
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    f()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.reps
                sp, _ = ops.decode_split_plan(b, a.hkv, ctx, bs, bt.shape[1], t)
                cells.append(f"{us:7.1f}us/{kv_bytes / us / 1e6:4.2f}TB s{sp:<2d}")
            print(f"{b:4d} {ctx:5d} " + " ".join(f"{c:>16s}" for c in cells), flush=True)
            del kc, vc
    ops.DECODE_TARGET_WAVES = 1024


if __name__ == "__main__":
    main()
