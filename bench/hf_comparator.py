"""Reference-equivalent single worker (BASELINE.md "Comparators"): HF transformers eager greedy
generation with PyTorch-ROCm on one MI355X, same model config (random init, no download),
same prompt/output lengths and batch as ``bench.py``.

The reference's only compute is ``torch.matmul`` on placeholder shards and its master/worker
path does not run, so this is the closest runnable stand-in for "the reference on
this hardware": what a user of the reference's loader (``src/model/loader.py:19-23``) gets from
``transformers`` directly.

    python bench/hf_comparator.py --model llama3-8b --batch 256 --prompt-len 128 --gen-len 128
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--prompt-len", type=int, default=128)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default="cuda")
    ap.add_argument("--attn", default="sdpa", help="transformers attn_implementation (sdpa | eager)")
    a = ap.parse_args()

    import torch
    import transformers
    from distributed_llms_amd.config import get_model_config

    cfg = get_model_config(a.model)
    hf_cfg = transformers.AutoConfig.for_model(**cfg.to_hf_config())
    hf_cfg._attn_implementation = a.attn
    torch.manual_seed(0)
    t0 = time.perf_counter()
    with torch.device(a.device):
        model = transformers.AutoModelForCausalLM.from_config(hf_cfg, torch_dtype=torch.bfloat16)
    model.eval()
    sync = torch.cuda.synchronize if a.device != "cpu" else (lambda: None)
    sync()
    load_s = time.perf_counter() - t0
    g = torch.Generator(device="cpu").manual_seed(0)
    ids = torch.randint(3, min(cfg.vocab_size, 30000), (a.batch, a.prompt_len), generator=g).to(a.device)
    mask = torch.ones_like(ids)
    kw = dict(attention_mask=mask, max_new_tokens=a.gen_len, min_new_tokens=a.gen_len, do_sample=False,
              pad_token_id=0, eos_token_id=None)

    with torch.inference_mode():
        for _ in range(a.warmup):
            model.generate(ids, **kw)
        sync()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            out = model.generate(ids, **kw)
        sync()
        el = time.perf_counter() - t0
    assert out.shape[1] == a.prompt_len + a.gen_len
    toks = a.steps * a.batch * a.gen_len
    print(json.dumps({"comparator": "hf-transformers-eager-generate", "transformers": transformers.__version__,
                      "torch": torch.__version__, "model": a.model, "batch": a.batch, "prompt_len": a.prompt_len,
                      "gen_len": a.gen_len, "attn": a.attn, "tokens_per_s": round(toks / el, 2),
                      "p50_latency_ms": round(1000 * el / a.steps, 1), "load_s": round(load_s, 1)}), flush=True)


if __name__ == "__main__":
    main()
