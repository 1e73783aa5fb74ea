"""Grouped expert prefill GEMMs in isolation (Mixtral-8x7B shapes): gemm_pp_moe vs the dense kernel.

    python bench/moe_prefill_bench.py [--tokens 32768] [--rounds 5]

T tokens routed top-2 over 8 experts with equal counts (T * 2 / 8 rows each), expert-sorted slots.
Candidates per projection (gate|up with the SwiGLU fused, then down), us per call and TF/s:
  pp_moe      gemm_pp_moe: one 256 x 256 tile per workgroup over the slot space, rows gathered
              through the slot -> token list inside the kernel
  (a persistent gemm_pf MOE form, with static and dynamic tile walks and 8 / 16 / 32-row-tile
  groups, was measured slower in round 5 -- profiles/round5_moe_prefill.md -- and removed)
  dense_pf    gemm_pf on ONE expert's weight over all slots: the same FLOPs, no expert segments
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd import _ext
from distributed_llms_amd.ops import gemm


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=32768)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    k = _ext.kernels()
    torch.manual_seed(0)
    E, H, I, top = 8, 4096, 14336, 2
    T = a.tokens
    slots = T * top
    per = slots // E
    counts = torch.full((E,), per, dtype=torch.int32, device="cuda")
    offsets = torch.arange(0, slots, per, dtype=torch.int32, device="cuda")[:E].contiguous()
    sorted_tok = torch.randperm(slots, device="cuda").remainder(T).to(torch.int32)
    x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
    xs = x.index_select(0, sorted_tok.long())
    wgu = torch.randn(E, 2 * I, H, device="cuda", dtype=torch.bfloat16) * 0.02
    wd = torch.randn(E, H, I, device="cuda", dtype=torch.bfloat16) * 0.02
    act = torch.empty(slots, I, device="cuda", dtype=torch.bfloat16)
    ys = torch.empty(slots, H, device="cuda", dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream

    def gu_pp():
        k.gemm_pp_moe(act.data_ptr(), x.data_ptr(), sorted_tok.data_ptr(), wgu.data_ptr(), counts.data_ptr(),
                      offsets.data_ptr(), E, 2 * I, H, T, slots, 1, st)

    def gu_dense():
        gemm.linear_pf(xs, wgu[0], swiglu=True)

    def dn_pp():
        k.gemm_pp_moe(ys.data_ptr(), act.data_ptr(), 0, wd.data_ptr(), counts.data_ptr(), offsets.data_ptr(),
                      E, H, I, slots, slots, 0, st)

    def dn_dense():
        gemm.linear_pf(act, wd[0])

    cands = {"gate_up": {"pp_moe": gu_pp, "dense_pf": gu_dense},
             "down": {"pp_moe": dn_pp, "dense_pf": dn_dense}}
    flops = {"gate_up": 2.0 * slots * 2 * I * H, "down": 2.0 * slots * H * I}
    for proj, fns in cands.items():
        res = {n: [] for n in fns}
        for fn in fns.values():
            fn()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for n, fn in fns.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                e1.synchronize()
                res[n].append(e0.elapsed_time(e1) * 1e3)
        cells = "  ".join(f"{n} {statistics.median(v):8.0f} us {flops[proj] / statistics.median(v) / 1e6:6.0f} TF/s"
                          for n, v in res.items())
        print(f"{proj:8s} T={T}: {cells}", flush=True)


if __name__ == "__main__":
    main()
