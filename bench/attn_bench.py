"""Paged decode attention microbenchmark (Llama-3 GQA shapes) on one MI355X.

Times N back-to-back launches between two events (the GPU never idles, so host launch
overhead is excluded) and reports us/call and KV bytes streamed per second, sweeping the
split-plan target (``knobs.attn_target_waves``).

    python bench/attn_bench.py [--batch 64 256] [--ctx 192 1024 4096]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import distributed_llms_amd.ops as ops
from distributed_llms_amd import knobs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[16, 64, 256])
    ap.add_argument("--ctx", type=int, nargs="+", default=[192, 1024, 4096])
    ap.add_argument("--targets", type=int, nargs="+", default=[512, 1024, 2048, 4096])
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--cold", action="store_true",
                    help="rotate over KV-cache copies totalling > 1 GB (every call streams from HBM, as in "
                         "the engine where each layer's KV is evicted by the weight stream); also time a "
                         "plain read of the same bytes (torch.sum) as the streaming reference")
    a = ap.parse_args()
    if a.cold:
        return cold(a)
    dev, bs = "cuda", 32
    print(f"{'B':>4s} {'ctx':>5s} " + " ".join(f"{'t' + str(t):>16s}" for t in a.targets))
    for b in a.batch:
        for ctx in a.ctx:
            mb = -(-ctx // bs) + 1
            nb = b * mb + 1
            kc = torch.randn(nb, a.hkv, bs, a.d, device=dev).to(torch.bfloat16)
            vc = torch.randn(nb, a.hkv, a.d, bs, device=dev).to(torch.bfloat16)
            perm = torch.randperm(nb - 1, device=dev)[: b * mb].to(torch.int32) + 1      # scattered blocks
            bt = perm.view(b, mb).contiguous()
            sl = torch.full((b,), ctx, dtype=torch.int32, device=dev)
            q = torch.randn(b, a.hq, a.d, device=dev).to(torch.bfloat16)
            kv_bytes = b * ctx * a.hkv * a.d * 2 * 2
            cells = []
            for t in a.targets:
                knobs.K.attn_target_waves = t
                f = lambda: ops.paged_attention_decode(q, kc, vc, bt, sl, 0.088, max_ctx=ctx)   # noqa: E731
                f()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    f()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) * 1e3 / a.reps
                sp, _ = ops.decode_split_plan(b, a.hkv, ctx, bs, bt.shape[1], t)
                cells.append(f"{us:7.1f}us/{kv_bytes / us / 1e6:4.2f}TB s{sp:<2d}")
            print(f"{b:4d} {ctx:5d} " + " ".join(f"{c:>16s}" for c in cells), flush=True)
            del kc, vc
    knobs.K.attn_target_waves = 1024


def cold(a):
    dev, bs = "cuda", 32
    print(f"{'B':>4s} {'ctx':>5s} {'attn_us':>8s} {'TB/s':>6s} {'fused_us':>8s} {'TB/s':>6s} {'sum_us':>8s} "
          f"{'TB/s':>6s}   (cold: rotating KV copies; fused = RoPE + KV append + attention from raw qkv)")
    for b in a.batch:
        for ctx in a.ctx:
            mb = -(-ctx // bs) + 1
            nb = b * mb + 1
            kv_bytes = b * ctx * a.hkv * a.d * 2 * 2
            copies = max(2, -(-(1 << 30) // (2 * nb * a.hkv * bs * a.d * 2)))
            caches = []
            for _ in range(copies):
                kc = torch.randn(nb, a.hkv, bs, a.d, device=dev).to(torch.bfloat16)
                vc = torch.randn(nb, a.hkv, a.d, bs, device=dev).to(torch.bfloat16)
                caches.append((kc, vc))
            perm = torch.randperm(nb - 1, device=dev)[: b * mb].to(torch.int32) + 1
            bt = perm.view(b, mb).contiguous()
            sl = torch.full((b,), ctx, dtype=torch.int32, device=dev)
            q = torch.randn(b, a.hq, a.d, device=dev).to(torch.bfloat16)
            # the reference read: the same number of bytes, contiguous, from the same rotation
            flat = [(kc.view(-1)[: kv_bytes // 4], vc.view(-1)[: kv_bytes // 4]) for kc, vc in caches]

            def timed(fn):
                fn(0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(a.reps):
                    fn(i % copies)
                e1.record()
                e1.synchronize()
                return e0.elapsed_time(e1) * 1e3 / a.reps
            t_attn = timed(lambda i: ops.paged_attention_decode(q, caches[i][0], caches[i][1], bt, sl, 0.088,
                                                                max_ctx=ctx))
            t_sum = timed(lambda i: (flat[i][0].sum(dtype=torch.float32), flat[i][1].sum(dtype=torch.float32)))
            from distributed_llms_amd.ops import reference as ref
            qkv = torch.randn(b, (a.hq + 2 * a.hkv) * a.d, device=dev).to(torch.bfloat16)
            pos = (sl - 1).contiguous()
            slots = (bt[torch.arange(b, device=dev), (ctx - 1) // bs] * bs + (ctx - 1) % bs).to(torch.int32)
            cs = ref.rope_cos_sin(a.d, 8192, 500000.0, device=dev)
            t_fused = timed(lambda i: ops.paged_attention_decode_rope(qkv, pos, cs, caches[i][0], caches[i][1], slots,
                                                                      bt, sl, a.hq, a.hkv, a.d, 0.088, max_ctx=ctx))
            t_nr = timed(lambda i: ops.paged_attention_decode_rope(qkv, pos, None, caches[i][0], caches[i][1], slots,
                                                                   bt, sl, a.hq, a.hkv, a.d, 0.088, max_ctx=ctx))
            t_sep = timed(lambda i: ops.paged_attention_decode(
                ops.rope_cache_append(qkv, pos, cs, caches[i][0], caches[i][1], slots, a.hq, a.hkv, a.d),
                caches[i][0], caches[i][1], bt, sl, 0.088, max_ctx=ctx))
            print(f"      fused without RoPE {t_nr:.1f} us, rope_cache + attention (two launches) {t_sep:.1f} us")
            print(f"{b:4d} {ctx:5d} {t_attn:8.1f} {kv_bytes / t_attn / 1e6:6.2f} {t_fused:8.1f} "
                  f"{kv_bytes / t_fused / 1e6:6.2f} {t_sum:8.1f} {kv_bytes / t_sum / 1e6:6.2f}", flush=True)
            del caches, flat


if __name__ == "__main__":
    main()
