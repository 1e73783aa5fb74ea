"""Cycle stamps inside gemm_pp (diagnostic build, variant bit 3): where a workgroup's time goes.

Per wave: main-loop cycles, cycles spent in the once-per-K-tile block B_t (counted vmcnt wait for
the next K-tile's LDS-DMA + s_barrier) and K-tiles; the rest of the loop is the MFMA stream with
its counted LDS waits.  Ideal MFMA time per K-tile = 2 x RT x CT x 16 cycles
(v_mfma_f32_16x16x32_bf16).  The kernel time of the normal build is printed beside it, and the
sum of workgroup loop spans / 256 CUs (what the loops alone would take if the CUs never idled).

    python bench/pp_stamps.py
"""
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd.ops import gemm

CASES = [  # name, M, N, K, swiglu, splits, variant (| 64: schedule 2, | 16 / 32: schedule-1 ablations)
    ("gate_up dec S2", 256, 28672, 4096, True, 2, 64), ("gate_up dec", 256, 28672, 4096, True, 1, 1),
    ("gate pf S2", 8192, 14336, 4096, False, 1, 68), ("gate pf", 8192, 14336, 4096, False, 1, 4),
    ("gate pf S2 BN128", 8192, 14336, 4096, False, 1, 69),
]


def timed(fn, it=10):
    ts = []
    for _ in range(it):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    return statistics.median(ts)


def main():
    torch.manual_seed(0)
    dev = torch.device("cuda")
    for name, m, n, k, sw, s, v in CASES:
        copies = max(1, -(-(768 << 20) // (n * k * 2))) if m <= 256 else 1
        ws_ = [(torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16) for _ in range(copies)]
        x = torch.randn(m, k, device=dev).to(torch.bfloat16)
        it = iter(range(10 ** 9))

        def run(var):
            return gemm.linear_pp(x, ws_[next(it) % copies], splits=s, swiglu=sw, variant=var)
        for _ in range(10):
            run((v & 7) | 8 | (v & 112))
        torch.cuda.synchronize()
        bn = 128 if v & 1 else 256
        # ablations time the diagnostic build itself (their output is garbage)
        grid = (n // bn) * (-(-m // 256)) * s
        full = gemm._workspace(dev)[-grid * 512:].view(grid * 4, 128).cpu()
        rec = full[:, :4]
        tot, bt, nt, rt = rec[:, 0], rec[:, 1], rec[:, 2], rec[:, 3]
        b1, b3 = (full[:, 20] / tot).tolist(), (full[:, 21] / tot).tolist()
        rt_ns = rt * 10.0
        ghz = statistics.median((tot / rt_ns).tolist())
        ideal = 2 * 8 * (bn // 32) * 16
        per = (tot / nt).tolist()
        frac = (bt / tot).tolist()
        t_real = timed(lambda: run((v & 7) | (v & 64) | (8 | (v & 48) if v & 48 else 0)))
        wg_us = (rt_ns / 1e3).view(-1, 4).max(dim=1).values
        print(f"{name:12s} M={m:5d} N={n:5d} K={k:5d} S={s:2d} BN={bn} var={v}: kernel {t_real:7.1f} us "
              f"({2.0 * m * n * k / t_real / 1e6:5.0f} TF) | WG loop median {statistics.median(wg_us.tolist()):6.1f} us, "
              f"sum/256 {wg_us.sum().item() / 256:7.1f} us | clock {ghz:.2f} GHz | cycles/K-tile "
              f"{statistics.median(per):6.0f} (ideal {ideal}, {ideal / statistics.median(per) * 100:3.0f} %) | "
              f"barrier share {statistics.median(frac) * 100:4.1f} %"
              + (f" (IB1 {statistics.median(b1) * 100:.1f} %, IB3 {statistics.median(b3) * 100:.1f} %)" if v & 64 else ""),
              flush=True)
        del ws_, x
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
