"""Token sampling on the last stage.

Greedy rows use the argmax kernel (K10 tail) on bf16 logits; rows with temperature > 0
use softmax + top-k/top-p + multinomial in torch (fp32).
"""
from __future__ import annotations

from typing import Optional, Sequence as Seq

import torch

from .. import ops


def sample(logits: torch.Tensor, temperatures: Optional[Seq[float]] = None, top_k: Optional[Seq[int]] = None,
           top_p: Optional[Seq[float]] = None, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    """logits [B, V] -> ids [B] int32 (device)."""
    if temperatures is None or all(t <= 0 for t in temperatures):
        return ops.argmax(logits)
    greedy = ops.argmax(logits)
    temps = torch.tensor([max(t, 1e-5) for t in temperatures], device=logits.device, dtype=torch.float32)
    lf = logits.float() / temps.unsqueeze(1)
    if top_k is not None and any(k > 0 for k in top_k):
        # one batched mask: row i keeps logits >= its k-th largest (k <= 0: every logit)
        kmax = min(max(top_k), lf.shape[1])
        vals, _ = torch.topk(lf, kmax, dim=-1)
        ks = torch.tensor(list(top_k), device=lf.device)
        thresh = vals.gather(1, (ks.clamp(1, kmax) - 1).unsqueeze(1))
        thresh = thresh.masked_fill((ks <= 0).unsqueeze(1), float("-inf"))
        lf = lf.masked_fill(lf < thresh, float("-inf"))
    probs = torch.softmax(lf, dim=-1)
    if top_p is not None and any(p < 1.0 for p in top_p):
        sp, si = torch.sort(probs, dim=-1, descending=True)
        cum = sp.cumsum(-1)
        tp = torch.tensor(list(top_p), device=logits.device).unsqueeze(1)
        mask = (cum - sp) > tp
        sp = sp.masked_fill(mask, 0.0)
        probs = torch.zeros_like(probs).scatter_(-1, si, sp)
        probs = probs / probs.sum(-1, keepdim=True)
    drawn = torch.multinomial(probs, 1, generator=generator).squeeze(1).to(torch.int32)
    is_greedy = torch.tensor([t <= 0 for t in temperatures], device=logits.device)
    return torch.where(is_greedy, greedy, drawn)


def step_sampling_args(seqs) -> dict:
    temps = [s.params.temperature for s in seqs]
    if all(t <= 0 for t in temps):
        return {}
    return {"temperatures": temps, "top_k": [s.params.top_k for s in seqs],
            "top_p": [s.params.top_p for s in seqs]}
