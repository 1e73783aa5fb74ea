"""End-to-end GPU correctness at production shapes: the exact B = 256 dispatch of the benchmark
(two 16K-token prefill steps, then HIP-graph-replayed decode) on layers of the real model dims,
checked against an fp32 PyTorch forward of the same (bf16-rounded) weights.

* Llama-3-8B dims (H 4096, I 14336, GQA 32 / 8 x 128, full 128,256-row LM head), 4 layers and 16
  graph-replayed decode steps: the
  wide / 256 x 256 GEMMs with f16 split-K slabs deferred into the add + RMSNorm kernels, the
  split-K qkv consumed by the fused RoPE + paged-attention decode kernel, the LM head GEMM and the
  graph bucket for 256 sequences.
* Mixtral-8x7B dims, 1 MoE layer: router, expert grouped GEMMs and combine at T = 4096 (prefill)
  and T = 256 (decode).

The fp32 reference recomputes the whole sequence every step (no KV cache), so it shares nothing
with the engine but the weights and the token ids; decode steps feed both sides the tokens the
engine picked.  Logits must agree to a fraction of their spread, and every row whose reference
top-2 gap exceeds twice the row's logit error must pick the same token.
"""
import dataclasses
import json
import os

import pytest
import torch
import torch.nn.functional as F

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.batch import build_host_batch
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.models.stage import ModelStage
from distributed_llms_amd.ops import reference as ref

pytestmark = pytest.mark.gpu

BATCH = 256


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _bf(t):
    return t.to(torch.bfloat16).float()


def _ref_logits(stage: ModelStage, w32, toks: torch.Tensor, chunk: int = 32, rnd=None) -> torch.Tensor:
    """fp32 forward of ``toks`` [B, T] (all positions, causal); last-position logits [B, V].
    ``rnd``: applied to every op's output -- ``_bf`` gives the bf16-storage / fp32-compute forward
    (what an exact bf16 kernel stack would produce): its distance from the fp32 one is the error
    floor of bf16 activations."""
    r = rnd or (lambda t: t)
    cfg = stage.cfg
    hq, hkv, d, eps = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, cfg.norm_eps
    out, margin = [], []
    for b0 in range(0, toks.shape[0], chunk):
        t = toks[b0:b0 + chunk]
        b, n = t.shape
        pos = torch.arange(n, device=t.device).repeat(b)
        x = w32["embed"][t]
        gap = torch.full((b,), float("inf"), device=t.device)
        for lw in w32["layers"]:
            h = r(_rms(x, lw["attn_norm"], eps))
            qkv = r(h @ lw["wqkv"].t()).view(b * n, hq + 2 * hkv, d)
            q = r(ref.apply_rope(qkv[:, :hq], pos, stage.cos_sin)).view(b, n, hq, d).transpose(1, 2)
            k = r(ref.apply_rope(qkv[:, hq:hq + hkv], pos, stage.cos_sin)).view(b, n, hkv, d).transpose(1, 2)
            v = qkv[:, hq + hkv:].reshape(b, n, hkv, d).transpose(1, 2)
            k = k.repeat_interleave(hq // hkv, dim=1)
            v = v.repeat_interleave(hq // hkv, dim=1)
            a = r(F.scaled_dot_product_attention(q, k, v, is_causal=True, scale=stage.scale))
            x = r(x + a.transpose(1, 2).reshape(b, n, hq * d) @ lw["wo"].t())
            h = r(_rms(x, lw["mlp_norm"], eps)).view(b * n, -1)
            if cfg.is_moe:
                probs = torch.softmax(h @ lw["router"].t(), dim=-1)
                top = probs.view(b, n, -1)[:, -1].topk(cfg.experts_per_token + 1, dim=-1).values
                gap = torch.minimum(gap, top[:, -2] - top[:, -1])    # routing margin, last position
                tw, ids = torch.topk(probs, cfg.experts_per_token, dim=-1)
                tw = tw / tw.sum(-1, keepdim=True)
                y = torch.zeros_like(h)
                for e in range(cfg.num_experts):
                    tok, slot = (ids == e).nonzero(as_tuple=True)
                    if tok.numel():
                        gu = h[tok] @ lw["experts_gate_up"][e].t()
                        i = gu.shape[-1] // 2
                        ye = (F.silu(gu[:, :i]) * gu[:, i:]) @ lw["experts_down"][e].t()
                        y.index_add_(0, tok, ye * tw[tok, slot].unsqueeze(1))
            else:
                gu = h @ lw["w_gate_up"].t()
                i = gu.shape[-1] // 2
                y = r(F.silu(gu[:, :i]) * gu[:, i:]) @ lw["w_down"].t()
            x = r(x + y.view(b, n, -1))
        out.append(r(_rms(x[:, -1], w32["final_norm"], eps)) @ w32["lm_head"].t())
        margin.append(gap)
    return torch.cat(out), torch.cat(margin)


def _check(got: torch.Tensor, ref_out, what: str, max_rel: float, mean_rel: float):
    """``ref_out`` = (fp32 logits, routing margin per row: the fp32 router-probability gap between
    the k-th and (k+1)-th expert, inf for dense models).  A row whose expert choice is close to a
    tie may legitimately route differently from bf16 activations and then differs by O(1): such
    rows may exceed the error bound only if their margin is small (< 0.02) and they are few
    (<= 5 %).  Every other row must meet it."""
    want, margin = ref_out
    got, want = got.float(), want.float()
    spread = want.std().item()
    err = (got - want).abs()
    row_err = err.max(dim=-1).values
    bad = row_err > max_rel * spread
    print(f"{what}: spread {spread:.4f} max err {err.max().item() / spread:.4f} mean err "
          f"{err.mean().item() / spread:.5f} (x spread); rows over the bound {int(bad.sum())}, their routing "
          f"margins {[round(float(x), 4) for x in margin[bad].tolist()]}", flush=True)
    assert bool((margin[bad] < 0.02).all()), (what, "rows off with a clear routing decision",
                                              row_err[bad].tolist(), margin[bad].tolist())
    assert int(bad.sum()) <= 0.05 * got.shape[0], (what, int(bad.sum()))
    assert err[~bad].mean().item() <= mean_rel * spread, (what, err[~bad].mean().item(), spread)
    top2 = want.topk(2, dim=-1).values
    decided = ((top2[:, 0] - top2[:, 1]) > 2 * row_err) & ~bad
    agree = got.argmax(-1) == want.argmax(-1)
    _record({"check": what, "spread": spread, "max_err_rel": err.max().item() / spread,
             "mean_err_rel": err.mean().item() / spread, "rows_over_bound": int(bad.sum()),
             "argmax_agree": float(agree.float().mean()), "bound_max_rel": max_rel, "bound_mean_rel": mean_rel})
    assert bool(agree[decided].all()), (what, int((~agree[decided]).sum()), int(decided.sum()))
    return float(agree.float().mean())


def _record(row):
    """Achieved errors of every check, one JSON line each, appended to the file named by
    DLLM_RECORD_ERRORS (unset: nothing is written; profiles/production_shape_errors.md holds the
    recorded table -- the 8B / Mixtral bounds sit ~1.2-1.3x above its max and mean, the 70B ones
    ~1.4x)."""
    path = os.environ.get("DLLM_RECORD_ERRORS")
    if not path:
        return
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "a") as f:
        f.write(json.dumps(row) + "\n")


def _run(model: str, layers: int, prompt_len: int, decode_steps: int, max_rel: float, mean_rel: float):
    cfg = dataclasses.replace(get_model_config(model), num_layers=layers)
    stage = ModelStage(cfg, 0, layers, "cuda", torch.bfloat16).init_synthetic(seed=11)
    w32 = {"layers": [{k: v.float() for k, v in lw.items()} for lw in stage.layers],
           "embed": stage.embed["embed"].float(), "final_norm": stage.head["final_norm"].float(),
           "lm_head": stage.lm_head_weight().float()}
    per_seq = -(-(prompt_len + decode_steps + 1) // 32)
    # prefill-first (no mixed steps): two whole 16K-token prefill steps, then decode
    eng = LLMEngine(EngineConfig(model=model, dtype="bfloat16", device="cuda", max_batch=BATCH, max_seq_len=512,
                                 num_kv_blocks=BATCH * per_seq + 8, graph_batch_sizes=(BATCH,),
                                 mixed_prefill_tokens=0), stage)
    g = torch.Generator().manual_seed(3)
    prompts = torch.randint(3, cfg.vocab_size, (BATCH, prompt_len), generator=g)
    seqs = [eng.add_request(p.tolist(), SamplingParams(max_new_tokens=decode_steps + 1, ignore_eos=True))
            for p in prompts]
    row_of = {s.seq_id: i for i, s in enumerate(seqs)}
    toks = prompts.cuda()
    logits = torch.empty(BATCH, cfg.vocab_size, dtype=torch.float32, device="cuda")
    n_prefill = 0
    while n_prefill < BATCH:                       # 16K-token prefill steps (the bench's chunking)
        st = eng.scheduler.schedule(0)
        assert st is not None and st.is_prefill
        out = eng.runner.execute(build_host_batch(st, eng.bm, 32))
        rows = torch.tensor([row_of[s.seq_id] for s in st.seqs], device="cuda")
        logits[rows] = out.float()
        eng.scheduler.complete(st, out.argmax(-1).tolist())
        n_prefill += len(st.seqs)
    ref32 = _ref_logits(stage, w32, toks)
    agree = [_check(logits, ref32, f"{model} prefill", max_rel, mean_rel)]
    # the error floor of bf16 activations: an exact bf16-storage / fp32-compute forward against the
    # fp32 one.  Ours (bf16 activations, f16 split-K slabs, bf16 logits) stays within 1.35x of it
    floor = _ref_logits(stage, w32, toks, rnd=_bf)[0]
    want, spread = ref32[0], ref32[0].std().item()
    floor_mean = (floor - want).abs().mean().item() / spread
    ours_mean = (logits - want).abs().mean().item() / spread
    print(f"{model} prefill: mean err / spread {ours_mean:.5f}; bf16-activation floor {floor_mean:.5f} "
          f"({ours_mean / floor_mean:.2f}x)", flush=True)
    _record({"check": f"{model} prefill bf16 floor", "mean_err_rel": floor_mean, "ours_mean_err_rel": ours_mean})
    if not cfg.is_moe:                 # MoE: near-tie routing rows differ by O(1) in either forward
        assert ours_mean <= 1.35 * floor_mean, (ours_mean, floor_mean)
    for step in range(decode_steps):
        toks = torch.cat([toks, logits.argmax(-1, keepdim=True)], dim=1)
        st = eng.scheduler.schedule(0)
        assert st is not None and not st.is_prefill and len(st.seqs) == BATCH
        out = eng.runner.execute(build_host_batch(st, eng.bm, 32)).float()   # graph replay (static output)
        rows = torch.tensor([row_of[s.seq_id] for s in st.seqs], device="cuda")
        logits = torch.empty_like(logits)
        logits[rows] = out
        eng.scheduler.complete(st, out.argmax(-1).int().cpu().numpy())
        agree.append(_check(logits, _ref_logits(stage, w32, toks), f"{model} decode {step}", max_rel, mean_rel))
    assert eng.runner.graphs is not None and eng.runner.graphs.graphs, "decode never replayed a graph"
    assert min(agree) >= 0.9, agree
    return agree


@pytest.mark.slow
def test_llama3_8b_dims_b256_prefill_and_graph_decode_vs_fp32(cuda):
    """4 layers, 16 graph-replayed decode steps."""
    _run("llama3-8b", layers=4, prompt_len=128, decode_steps=16, max_rel=0.15, mean_rel=0.02)


@pytest.mark.slow
def test_llama3_70b_dims_layer_b256_vs_fp32(cuda):
    """One Llama-3-70B layer (H 8192, I 28672, 64 / 8 heads) through the default dispatch: the
    K = 8192 qkv / o projections ("proj" rule: N >= K, not the down-projection path), the 57344 x
    8192 gate|up, the 8192 x 28672 down, and the 128,256-row LM head at H = 8192."""
    _run("llama3-70b", layers=1, prompt_len=64, decode_steps=4, max_rel=0.1, mean_rel=0.013)


@pytest.mark.slow
def test_mixtral_dims_moe_layer_b256_vs_fp32(cuda):
    _run("mixtral-8x7b", layers=1, prompt_len=16, decode_steps=3, max_rel=0.15, mean_rel=0.02)
