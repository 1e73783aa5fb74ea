"""GEMM kernels for rocprofv3 counter passes (scripts/gpu_gemm_counters.sh), a few dispatches
each.  GCTR=decode: the decode MLP gate|up (M = 256, SwiGLU) and the o projection (split-K) on
gemm_wide.  (The round-4 gemm_rw rows of profiles/round4_gemm_counters.md came from the same
script with that kernel in the tree.)  GCTR=prefill: a prefill
projection (T = 8192, N = 6144, K = 4096) on gemm_pf, gemm_pp schedule 2 and hipBLASLt."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from distributed_llms_amd.ops import gemm


def main():
    torch.manual_seed(0)
    bf = lambda *s, sc=1.0: (torch.randn(*s, device="cuda") * sc).to(torch.bfloat16)   # noqa: E731
    mode = os.environ.get("GCTR", "decode")
    if mode == "decode":
        xd = bf(256, 4096)
        wgu = [bf(28672, 4096, sc=0.02) for _ in range(4)]    # > L2 / MALL reuse between calls
        wo = [bf(4096, 4096, sc=0.02) for _ in range(4)]
        for i in range(4):
            gemm.linear_wide(xd, wgu[i % 4], swiglu=True)
            gemm.linear_wide(xd, wo[i % 4], defer=True)
    else:
        x, w = bf(8192, 4096), bf(6144, 4096, sc=0.02)
        for _ in range(4):
            gemm.linear_pf(x, w)
            gemm.linear_pp(x, w, splits=1, variant=gemm.PP_PREFILL_VARIANT)
            F.linear(x, w)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
