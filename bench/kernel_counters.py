"""Run each hand-written HIP kernel a few times at Llama-3-8B decode shapes (B=256), for
rocprofv3 counter collection (``scripts/gpu_counters.sh``, ``tests/test_counters_gpu.py``):

    rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d out -o run \\
        --output-format csv -- python bench/kernel_counters.py

Kernels: wide decode GEMMs (down projection with deferred f16 split-K slabs, MLP up + SwiGLU,
LM head), fused split-K reduce + add + RMSNorm, paged decode attention, LDS-ring prefill
attention, RoPE + KV append, RMSNorm, SwiGLU, MoE router + MFMA grouped expert GEMM, argmax.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

import distributed_llms_amd.ops as ops
from distributed_llms_amd.ops import gemm, moe
from distributed_llms_amd.ops import reference as ref


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", default="", help="comma list: gemm,gate_up,lm_head,attn,prefill,rope,norm,silu,moe,argmax")
    a = ap.parse_args()
    only = set(x for x in a.only.split(",") if x)
    want = lambda k: not only or k in only   # noqa: E731
    dev = "cuda"
    torch.manual_seed(0)
    bf = lambda *s, sc=1.0: (torch.randn(*s, device=dev) * sc).to(torch.bfloat16)   # noqa: E731
    m, h, inter = 256, 4096, 14336
    for _ in range(a.reps):
        if want("gemm"):
            x, w = bf(m, inter, sc=0.5), bf(h, inter, sc=0.02)
            p = gemm.linear_wide(x, w, defer=True)
            res, g = bf(m, h), bf(h)
            if want("norm"):
                ops.fused_add_rms_norm(p, res, g, 1e-5)
            else:
                p.materialize()
        if want("gate_up"):
            gemm.linear_wide(bf(m, h, sc=0.5), bf(2 * inter, h, sc=0.02), swiglu=True)
        if want("lm_head"):
            gemm.linear_wide(bf(m, h, sc=0.5), bf(128256, h, sc=0.02))
        if want("norm"):
            ops.fused_add_rms_norm(bf(m, h), bf(m, h), bf(h), 1e-5)
        if want("silu"):
            ops.silu_mul(bf(m, 2 * inter))
        if want("attn"):
            b, hq, hkv, d, bs, ctx = 256, 32, 8, 128, 32, 192
            mb = ctx // bs + 1
            kc, vc = bf(b * mb + 1, hkv, bs, d), bf(b * mb + 1, hkv, d, bs)
            bt = (torch.randperm(b * mb, device=dev).to(torch.int32) + 1).view(b, mb)
            ops.paged_attention_decode(bf(b, hq, d), kc, vc, bt, torch.full((b,), ctx, dtype=torch.int32, device=dev),
                                       0.088, max_ctx=ctx)
        if want("prefill"):
            b, L, hq, hkv, d, bs = 256, 128, 32, 8, 128, 32
            nb = L // bs
            kc, vc = bf(b * nb + 1, hkv, bs, d), bf(b * nb + 1, hkv, d, bs)
            bt = (torch.arange(b * nb, device=dev, dtype=torch.int32) + 1).view(b, nb)
            cu = torch.arange(0, (b + 1) * L, L, dtype=torch.int32, device=dev)
            ops.paged_attention_prefill(bf(b * L, hq, d), kc, vc, bt, cu,
                                        torch.full((b,), L, dtype=torch.int32, device=dev), 0.088)
        if want("rope"):
            hq, hkv, d, bs = 32, 8, 128, 32
            kc = torch.zeros(8 * m + 64, hkv, bs, d, dtype=torch.bfloat16, device=dev)
            vc = torch.zeros(8 * m + 64, hkv, d, bs, dtype=torch.bfloat16, device=dev)
            cs = ref.rope_cos_sin(d, 4096, 500000.0, None).to(dev)
            ops.rope_cache_append(bf(m, (hq + 2 * hkv) * d), torch.full((m,), 161, dtype=torch.int32, device=dev), cs,
                                  kc, vc, (torch.arange(m, device=dev, dtype=torch.int32) * 7 + 3) * bs + 1,
                                  hq, hkv, d)
        if want("moe"):
            t, e = 256, 8
            moe.forward(bf(t, h), bf(e, h, sc=0.02), bf(e, 2 * inter, h, sc=0.02), bf(e, h, inter, sc=0.02), 2)
        if want("argmax"):
            ops.argmax(bf(m, 128256))
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
