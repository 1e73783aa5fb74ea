"""Grouped expert prefill GEMMs in isolation (Mixtral-8x7B shapes): why is the persistent form slower?

    python bench/moe_prefill_bench.py [--tokens 32768] [--rounds 5]

T tokens routed top-2 over 8 experts with equal counts (T * 2 / 8 rows each), expert-sorted slots.
Candidates per projection (gate|up with the SwiGLU fused, then down), us per call and TF/s:
  pp_moe      gemm_pp_moe: one 256 x 256 tile per workgroup over the slot space, rows gathered
              through the slot -> token list inside the kernel
  pf_moe      gemm_pf MOE form, static tile walk (rows pre-gathered into slot order)
  pf_moe_dyn  the same with the per-XCD dynamic tile queue
  pf_moe_g32 / _g16   static walk with 32 / 16 row tiles per group of the tile order (8 default):
              a group spanning an expert's whole segment reads its weight once
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

    def gu_pf(walk):
        return lambda: k.gemm_pf_moe(act.data_ptr(), xs.data_ptr(), wgu.data_ptr(), counts.data_ptr(),
                                     offsets.data_ptr(), E, 2 * I, H, slots, 1 | walk, st)

    def gu_dense():
        gemm.linear_pf(xs, wgu[0], swiglu=True)

    def dn_pp():
        k.gemm_pp_moe(ys.data_ptr(), act.data_ptr(), 0, wd.data_ptr(), counts.data_ptr(), offsets.data_ptr(),
                      E, H, I, slots, slots, 0, st)

    def dn_pf(walk):
        return lambda: k.gemm_pf_moe(ys.data_ptr(), act.data_ptr(), wd.data_ptr(), counts.data_ptr(),
                                     offsets.data_ptr(), E, H, I, slots, walk, st)

    def dn_dense():
        gemm.linear_pf(act, wd[0])

    cands = {"gate_up": {"pp_moe": gu_pp, "pf_moe": gu_pf(2), "pf_moe_dyn": gu_pf(0), "pf_moe_g32": gu_pf(2 | 4),
                         "pf_moe_g16": gu_pf(2 | 8), "dense_pf": gu_dense},
             "down": {"pp_moe": dn_pp, "pf_moe": dn_pf(2), "pf_moe_dyn": dn_pf(0), "pf_moe_g32": dn_pf(2 | 4),
                      "pf_moe_g16": dn_pf(2 | 8), "dense_pf": dn_dense}}
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
