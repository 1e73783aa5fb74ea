"""Would splitting the LM head between the last and the first pipeline stage balance pp8?

Evaluates the calibrated decode-time model of parallel/planner.py (half-layer units; MI355X,
Llama-3-8B, batch 256, context 192; pp8 modelled 1.0829 vs measured 1.0834 max/mean,
profiles/pp_stage_balance.md) with a fraction f of the LM head (and a combine cost) moved to
stage 0, re-partitioned by the same exact min-max DP.

    python bench/pp_head_split_model.py [--model llama3-8b] [--combine-us 8]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from distributed_llms_amd.config import get_model_config
from distributed_llms_amd.parallel import planner as P


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--combine-us", type=float, default=8.0)
    a = ap.parse_args()
    cfg = get_model_config(a.model)
    costs, head = P.unit_costs_us(cfg, 256, 192)
    print(f"{a.model}: {len(costs)} half-layer units, attention {costs[0]:.1f} us, MLP {costs[1]:.1f} us, "
          f"LM head {head:.1f} us")
    for n in (2, 4, 8):
        for f in (0.0, 0.25, 0.5, 0.75):
            fe = f * head + (a.combine_us if f > 0 else 0.0)
            units = P._partition(costs, n, head * (1 - f), first_extra=fe)
            pre = [0.0]
            for c in costs:
                pre.append(pre[-1] + c)
            cs = [pre[b] - pre[a_] + (fe if k == 0 else 0) + (head * (1 - f) if k == n - 1 else 0)
                  for k, (a_, b) in enumerate(units)]
            print(f"pp{n} head on stage 0: {f:4.2f}  stages {[round(c) for c in cs]}  "
                  f"max/mean {max(cs) / (sum(cs) / n):.4f}")


if __name__ == "__main__":
    main()
