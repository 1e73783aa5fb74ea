"""Offline hipBLASLt solution selection (PyTorch TunableOp) for every library GEMM shape the
engine issues, written to an in-tree CSV that the engine loads read-only at start-up
(``distributed_llms_amd/ops/tuning.py``).

Shapes per model: the decode graph buckets (M = EngineConfig.graph_batch_sizes) and the prefill
chunk (M = --prefill-tokens) for qkv / o / gate_up / down, plus the LM head at every decode
bucket.  Shapes the engine routes to its own HIP kernels are tuned anyway (cheap) so the
library fallback (kernel knob wide=none) is tuned too.

    python bench/tune_gemms.py --models llama3-8b llama3-70b mixtral-8x7b
"""
import argparse
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "distributed_llms_amd", "tuning",
                   "tunableop_gfx950.csv")


def shapes(model: str):
    from distributed_llms_amd.config import get_model_config
    c = get_model_config(model)
    hd = c.head_dim
    out = {"qkv": ((c.num_heads + 2 * c.num_kv_heads) * hd, c.hidden_size), "o": (c.hidden_size, c.num_heads * hd),
           "lm_head": (c.vocab_size, c.hidden_size)}
    if not c.is_moe:
        out["gate_up"] = (2 * c.intermediate_size, c.hidden_size)
        out["down"] = (c.hidden_size, c.intermediate_size)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", nargs="+", default=["llama3-8b", "llama3-70b", "mixtral-8x7b"])
    ap.add_argument("--decode-batches", type=int, nargs="+",
                    default=[1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192, 256, 384, 512])
    ap.add_argument("--prefill-tokens", type=int, nargs="*", default=[16384, 32768])
    ap.add_argument("--rotating-mb", type=int, default=0,
                    help="TunableOp rotating buffer (MB): operands cycle so a weight is never timed warm from the "
                         "256 MB Infinity Cache.  Measured end to end it did not help (Llama-3-8B B=256: 23.3k "
                         "tok/s with a 512 MB buffer vs 23.4k with the warm-tuned table), so it is off")
    ap.add_argument("--max-ms", type=int, default=30, help="per-solution tuning budget")
    ap.add_argument("--out", default=OUT)
    ap.add_argument("--merge", default=None, metavar="CSV",
                    help="start from this table (its results are kept; only new shapes are tuned)")
    ap.add_argument("--skip-decode", action="store_true", help="tune only the --prefill-tokens shapes")
    a = ap.parse_args()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    tmp = a.out + ".tmp%d.csv"     # TunableOp's own end-of-process dump (discarded)
    tun = torch.cuda.tunable
    tun.set_filename(tmp)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_max_tuning_iterations(30)
    if a.rotating_mb:
        tun.set_rotating_buffer_size(a.rotating_mb)
    tun.enable(True)
    if a.merge:
        assert tun.read_file(a.merge), f"could not load {a.merge}"
        print(f"loaded {len(tun.get_results())} results from {a.merge}", flush=True)
    tun.tuning_enable(True)
    t0 = time.time()
    seen = set()
    for model in a.models:
        for name, (n, k) in shapes(model).items():
            w = (torch.randn(n, k, device="cuda") * 0.02).to(torch.bfloat16)
            ms = ([] if a.skip_decode else list(a.decode_batches)) + ([] if name == "lm_head" else list(a.prefill_tokens))
            for m in ms:
                if (m, n, k) in seen:
                    continue
                seen.add((m, n, k))
                x = torch.randn(m, k, device="cuda").to(torch.bfloat16)
                F.linear(x, w)
                torch.cuda.synchronize()
                print(f"[{time.time() - t0:7.1f}s] tuned {model:13s} {name:8s} M={m:6d} N={n:6d} K={k:6d}", flush=True)
            del w
            torch.cuda.empty_cache()
    tun.tuning_enable(False)
    # TunableOp only flushes its file at C++ teardown; write the same CSV format ourselves
    vals = tun.get_validators()
    res = tun.get_results()
    with open(a.out, "w") as f:
        for kv in (vals.items() if hasattr(vals, "items") else vals):
            f.write(f"Validator,{kv[0]},{kv[1]}\n")
        for r in res:
            f.write(",".join(str(x) for x in r) + "\n")
    for g in glob.glob(a.out + ".tmp*"):
        os.remove(g)
    print(f"wrote {a.out}: {len(res)} results in {time.time() - t0:.0f}s", flush=True)

if __name__ == "__main__":
    main()
