"""Cycle stamps inside gemm_pp (diagnostic build, variant bit 3): where a K-tile's cycles go.

Per wave: loop cycles, cycles spent in the once-per-K-tile block B_t (counted vmcnt wait for the
next K-tile's LDS-DMA + s_barrier), and K-tiles; the rest of the loop is the MFMA stream with its
counted LDS waits.  Ideal MFMA time per K-tile = 2 x RT x CT x 16 cycles (v_mfma_f32_16x16x32_bf16).

    python bench/pp_stamps.py [--m 32768] [--n 14336] [--k 4096] [--variant 4]
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from distributed_llms_amd.ops import _ext


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[32768, 8192, 256])
    ap.add_argument("--n", type=int, default=14336)
    ap.add_argument("--k", type=int, default=4096)
    ap.add_argument("--variant", type=int, nargs="+", default=[4, 1, 5])
    a = ap.parse_args()
    torch.manual_seed(0)
    kern = _ext.kernels()
    w = (torch.randn(a.n, a.k, device="cuda") * 0.02).to(torch.bfloat16)
    for m in a.m:
        x = torch.randn(m, a.k, device="cuda").to(torch.bfloat16)
        y = torch.empty(m, a.n, dtype=torch.bfloat16, device="cuda")
        for v in a.variant:
            bn = 128 if v & 1 else 256
            grid = (a.n // bn) * ((m + 255) // 256)
            ws = torch.zeros(grid * 16, dtype=torch.float32, device="cuda")
            st = torch.cuda.current_stream().cuda_stream
            for _ in range(20):        # warm clocks; the last launch's stamps are read
                kern.gemm_pp(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, a.n, a.k, 1, 0,
                             v | 8, st)
            torch.cuda.synchronize()
            s = ws.view(-1, 4).cpu()

            def launch(var):
                kern.gemm_pp(y.data_ptr(), x.data_ptr(), w.data_ptr(), ws.data_ptr(), ws.numel(), m, a.n, a.k, 1, 0,
                             var, st)

            def time_us(var, it=10):
                ts = []
                for _ in range(it):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    launch(var)
                    e1.record()
                    e1.synchronize()
                    ts.append(e0.elapsed_time(e1) * 1e3)
                return statistics.median(ts)
            t_diag, t_real = time_us(v | 8), time_us(v)
            s2 = ws.view(-1, 4).cpu()
            wg_us = (s2[:, 3] * 10.0 / 1e3).view(-1, 4).max(dim=1).values
            print(f"   kernel us: diagnostic (no epilogue) {t_diag:.1f}, real {t_real:.1f}; grid {grid} WGs = "
                  f"{grid / 256:.2f} per CU; sum of WG loop spans / 256 = {wg_us.sum().item() / 256:.1f} us; "
                  f"TF real {2.0 * m * a.n * a.k / t_real / 1e6:.0f}", flush=True)
            tot, bt, nt, rt = s[:, 0], s[:, 1], s[:, 2], s[:, 3]
            rt_ns = rt * 10.0
            ghz = statistics.median((tot / rt_ns).tolist())
            rtile = 8 * (bn // 32)
            ideal = 2 * rtile * 16
            per = (tot / nt).tolist()
            frac = (bt / tot).tolist()
            print(f"M={m:6d} N={a.n} K={a.k} variant={v} BN={bn}: clock {ghz:.2f} GHz | cycles/K-tile median "
                  f"{statistics.median(per):7.0f} (ideal {ideal}, {ideal / statistics.median(per) * 100:.0f} %) "
                  f"p10 {sorted(per)[len(per) // 10]:.0f} p90 {sorted(per)[9 * len(per) // 10]:.0f} | B_t share "
                  f"median {statistics.median(frac) * 100:.1f} % p90 {sorted(frac)[9 * len(frac) // 10] * 100:.1f} % | "
                  f"loop us median {statistics.median(rt_ns.tolist()) / 1e3:.1f}", flush=True)


if __name__ == "__main__":
    main()
