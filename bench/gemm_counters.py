"""GEMM kernels for rocprofv3 counter passes (scripts/gpu_gemm_counters.sh): the ping-pong
kernel and hipBLASLt on one prefill shape, the wide and ping-pong kernels on the decode MLP
up projection, each a few dispatches."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from distributed_llms_amd.ops import gemm


def main():
    torch.manual_seed(0)
    bf = lambda *s, sc=1.0: (torch.randn(*s, device="cuda") * sc).to(torch.bfloat16)   # noqa: E731
    var = int(os.environ.get("PP_VAR", "4"))
    x, w = bf(8192, 4096), bf(14336, 4096, sc=0.02)
    xd, wd = bf(256, 4096), bf(28672, 4096, sc=0.02)
    decode_only = os.environ.get("DECODE_ONLY") == "1"
    for _ in range(4):
        if not decode_only:
            gemm.linear_pp(x, w, splits=1, variant=var)
            F.linear(x, w)
            gemm.linear_pp(xd, wd, splits=1, swiglu=True, variant=1 | 2)
        gemm.linear_wide(xd, wd, swiglu=True)
        gemm.linear_gate_up56(xd, wd, variant=0)
        gemm.linear_gate_up56(xd, wd, variant=1)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
