"""LM-head GEMM time vs how much HBM is already allocated (hipBLASLt workspace / algo choice)."""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from blas_graph_probe import t_eager, t_graph  # noqa: E402


def main():
    w = (torch.randn(128256, 4096, device="cuda") * 0.02).to(torch.bfloat16)
    x = torch.randn(128, 4096, device="cuda").to(torch.bfloat16)
    fn = lambda: F.linear(x, w)
    print("baseline eager/graph us:", round(t_eager(fn), 1), round(t_graph(fn), 1), flush=True)
    hogs = []
    for frac in (0.5, 0.8, 0.95):
        free, total = torch.cuda.mem_get_info()
        want = int(free * frac) - (1 << 30)
        if want > 0:
            hogs.append(torch.empty(want, dtype=torch.uint8, device="cuda"))
        free2, _ = torch.cuda.mem_get_info()
        print(f"after hogging {frac}: free {free2/2**30:.1f} GiB -> eager/graph us:",
              round(t_eager(fn), 1), round(t_graph(fn), 1), flush=True)
    torch.backends.cuda.preferred_blas_library("cublas")
    print("rocBLAS backend eager/graph us:", round(t_eager(fn), 1), round(t_graph(fn), 1), flush=True)


if __name__ == "__main__":
    main()
