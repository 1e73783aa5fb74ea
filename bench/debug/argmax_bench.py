"""argmax over the LM head's logits (B x 128256 bf16), us per call: the K10 tail of every decode step.

    python bench/debug/argmax_bench.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch

from distributed_llms_amd import ops


def main():
    for rows in (64, 256):
        xs = [torch.randn(rows, 128256, device="cuda").to(torch.bfloat16) for _ in range(8)]   # > L2 each round
        ops.argmax(xs[0])
        torch.cuda.synchronize()
        res = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(40):
                ops.argmax(xs[i % 8])
            e1.record()
            e1.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / 40)
        t = statistics.median(res)
        print(f"argmax rows={rows:4d} vocab=128256  {t:6.1f} us  ({rows * 128256 * 2 / t / 1e6:.2f} TB/s)", flush=True)


if __name__ == "__main__":
    main()
