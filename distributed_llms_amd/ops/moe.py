"""Mixtral MoE: router (K11) and expert MLPs (K12)."""
from __future__ import annotations

import torch

from . import reference as ref


def route(router_logits: torch.Tensor, top_k: int):
    return ref.moe_route(router_logits, top_k)


def mlp(x, w_gate_up, w_down, topk_w, topk_ids):
    return ref.moe_mlp(x, w_gate_up, w_down, topk_w, topk_ids)
