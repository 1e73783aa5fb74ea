"""Decode GEMM shapes: default hipBLASLt heuristic vs TunableOp-selected solution.

    PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_FILENAME=tunableop/llama3_8b.csv python bench/tunableop_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from blas_graph_probe import t_graph  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096)}


def main():
    ms = [int(x) for x in os.environ.get("PROBE_M", "64,128,256").split(",")]
    ws = {k: (torch.randn(n, kk, device="cuda") * 0.02).to(torch.bfloat16) for k, (n, kk) in SHAPES.items()}
    res = {}
    torch.cuda.tunable.enable(False)
    for name, w in ws.items():
        for m in ms:
            x = torch.randn(m, w.shape[1], device="cuda").to(torch.bfloat16)
            res[(name, m)] = [t_graph(lambda: F.linear(x, w))]
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    for name, w in ws.items():
        for m in ms:
            x = torch.randn(m, w.shape[1], device="cuda").to(torch.bfloat16)
            F.linear(x, w)                    # tune (eager)
            res[(name, m)].append(t_graph(lambda: F.linear(x, w)))
            n, k = SHAPES[name]
            t0, t1 = res[(name, m)]
            print(f"{name:8s} M={m:4d} default {t0:8.1f} us ({n*k*2/t0/1e6:5.2f} TB/s)   tuned {t1:8.1f} us "
                  f"({n*k*2/t1/1e6:5.2f} TB/s)  x{t0/t1:.2f}", flush=True)
    torch.cuda.tunable.write_file()


if __name__ == "__main__":
    main()
