"""Weight specs, HF <-> runtime name mapping, and seeded synthetic init.

Runtime layout (what the kernels consume) per transformer block:
  llama / mixtral: attn_norm [H], wqkv [(Hq+2Hkv)D, H] (q|k|v fused), wo [H, HqD], mlp_norm [H],
                   dense: w_gate_up [2I, H] (gate|up fused), w_down [H, I]
                   moe:   router [E, H], experts_gate_up [E, 2I, H], experts_down [E, H, I]
  gpt2:            ln1_w, ln1_b, wqkv [3H, H], bqkv, wo [H, H], bo, ln2_w, ln2_b,
                   w_fc [I, H], b_fc, w_proj [H, I], b_proj
Non-block tensors: embed [V, H] (+ pos_embed [P, H] for gpt2) on the first stage;
final_norm (+ final_norm_b) and lm_head [V, H] on the last stage (lm_head = embed when tied).

Checkpoints on disk keep HF parameter names (the reference's shards hold HF keys,
``src/model/shard_manager.py:30-67``), so ``reconstruct_model`` yields an HF state dict.

Synthetic init: every tensor is drawn from a generator seeded by (seed, layer, name), so a
layer's weights are identical whatever stage count / device split generates them.
"""
from __future__ import annotations

import re
import zlib
from typing import Dict, Iterable, List, Optional, Tuple

import torch

from ..config import ModelConfig

EMBED = -1       # pseudo layer index for embeddings
HEAD = -2        # pseudo layer index for final norm / lm head


def block_shapes(cfg: ModelConfig) -> Dict[str, Tuple[int, ...]]:
    h, i, d = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    if cfg.arch == "gpt2":
        return {
            "ln1_w": (h,), "ln1_b": (h,), "wqkv": (3 * h, h), "bqkv": (3 * h,), "wo": (h, h), "bo": (h,),
            "ln2_w": (h,), "ln2_b": (h,), "w_fc": (i, h), "b_fc": (i,), "w_proj": (h, i), "b_proj": (h,),
        }
    s = {"attn_norm": (h,), "wqkv": (cfg.qkv_size, h), "wo": (h, cfg.q_size), "mlp_norm": (h,)}
    if cfg.is_moe:
        e = cfg.num_experts
        s.update({"router": (e, h), "experts_gate_up": (e, 2 * i, h), "experts_down": (e, h, i)})
    else:
        s.update({"w_gate_up": (2 * i, h), "w_down": (h, i)})
    return s


def embed_shapes(cfg: ModelConfig) -> Dict[str, Tuple[int, ...]]:
    s = {"embed": (cfg.vocab_size, cfg.hidden_size)}
    if cfg.arch == "gpt2":
        s["pos_embed"] = (cfg.max_position, cfg.hidden_size)
    return s


def head_shapes(cfg: ModelConfig) -> Dict[str, Tuple[int, ...]]:
    s = {"final_norm": (cfg.hidden_size,)}
    if cfg.arch == "gpt2":
        s["final_norm_b"] = (cfg.hidden_size,)
    if not cfg.tie_embeddings:
        s["lm_head"] = (cfg.vocab_size, cfg.hidden_size)
    return s


def _is_norm(name: str) -> bool:
    return name in ("attn_norm", "mlp_norm", "final_norm", "ln1_w", "ln2_w")


def _is_bias(name: str) -> bool:
    return name.startswith("b") or name.endswith("_b")


def tensor_seed(seed: int, layer: int, name: str) -> int:
    return (seed * 1000003 + (layer + 7) * 7919 + zlib.crc32(name.encode())) & 0x7FFFFFFF


def synth_tensor(seed: int, layer: int, name: str, shape, dtype, device, std: float = 0.02) -> torch.Tensor:
    """Deterministic N(0, std) (norm weights = 1, biases = 0) generated directly on ``device``."""
    if _is_norm(name):
        return torch.ones(shape, dtype=dtype, device=device)
    if _is_bias(name) and name not in ("bqkv",):
        return torch.zeros(shape, dtype=dtype, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(tensor_seed(seed, layer, name))
    out = torch.empty(shape, dtype=dtype, device=device)
    # chunk along dim 0 to bound the fp32 temporary (70B/Mixtral expert tensors are GBs)
    rows = shape[0]
    per = max(1, (1 << 26) // max(1, int(torch.tensor(shape[1:]).prod().item()) if len(shape) > 1 else 1))
    for r0 in range(0, rows, per):
        r1 = min(rows, r0 + per)
        out[r0:r1] = (torch.randn((r1 - r0,) + tuple(shape[1:]), generator=g, device=device) * std).to(dtype)
    if name == "bqkv":
        out.mul_(0.5)
    return out


# ------------------------------------------------------------------ HF naming
def hf_block_names(cfg: ModelConfig, layer: int) -> List[str]:
    if cfg.arch == "gpt2":
        p = f"transformer.h.{layer}."
        return [p + n for n in ("ln_1.weight", "ln_1.bias", "attn.c_attn.weight", "attn.c_attn.bias",
                                "attn.c_proj.weight", "attn.c_proj.bias", "ln_2.weight", "ln_2.bias",
                                "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias")]
    p = f"model.layers.{layer}."
    names = [p + "input_layernorm.weight", p + "self_attn.q_proj.weight", p + "self_attn.k_proj.weight",
             p + "self_attn.v_proj.weight", p + "self_attn.o_proj.weight", p + "post_attention_layernorm.weight"]
    if cfg.is_moe:
        names.append(p + "block_sparse_moe.gate.weight")
        for e in range(cfg.num_experts):
            names += [p + f"block_sparse_moe.experts.{e}.{w}.weight" for w in ("w1", "w2", "w3")]
    else:
        names += [p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight", p + "mlp.down_proj.weight"]
    return names


def block_to_hf(cfg: ModelConfig, layer: int, w: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """Runtime block tensors -> HF-named state-dict entries."""
    if cfg.arch == "gpt2":
        p = f"transformer.h.{layer}."
        return {
            p + "ln_1.weight": w["ln1_w"], p + "ln_1.bias": w["ln1_b"],
            p + "attn.c_attn.weight": w["wqkv"].t().contiguous(), p + "attn.c_attn.bias": w["bqkv"],
            p + "attn.c_proj.weight": w["wo"].t().contiguous(), p + "attn.c_proj.bias": w["bo"],
            p + "ln_2.weight": w["ln2_w"], p + "ln_2.bias": w["ln2_b"],
            p + "mlp.c_fc.weight": w["w_fc"].t().contiguous(), p + "mlp.c_fc.bias": w["b_fc"],
            p + "mlp.c_proj.weight": w["w_proj"].t().contiguous(), p + "mlp.c_proj.bias": w["b_proj"],
        }
    p = f"model.layers.{layer}."
    q, k, v = torch.split(w["wqkv"], [cfg.q_size, cfg.kv_size, cfg.kv_size], 0)
    out = {p + "input_layernorm.weight": w["attn_norm"], p + "self_attn.q_proj.weight": q.contiguous(),
           p + "self_attn.k_proj.weight": k.contiguous(), p + "self_attn.v_proj.weight": v.contiguous(),
           p + "self_attn.o_proj.weight": w["wo"], p + "post_attention_layernorm.weight": w["mlp_norm"]}
    i = cfg.intermediate_size
    if cfg.is_moe:
        out[p + "block_sparse_moe.gate.weight"] = w["router"]
        for e in range(cfg.num_experts):
            q = p + f"block_sparse_moe.experts.{e}."
            out[q + "w1.weight"] = w["experts_gate_up"][e, :i].contiguous()
            out[q + "w3.weight"] = w["experts_gate_up"][e, i:].contiguous()
            out[q + "w2.weight"] = w["experts_down"][e].contiguous()
    else:
        out[p + "mlp.gate_proj.weight"] = w["w_gate_up"][:i].contiguous()
        out[p + "mlp.up_proj.weight"] = w["w_gate_up"][i:].contiguous()
        out[p + "mlp.down_proj.weight"] = w["w_down"]
    return out


def hf_to_block(cfg: ModelConfig, layer: int, sd: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
    """HF-named entries for one block -> runtime (fused) tensors."""
    if cfg.arch == "gpt2":
        p = f"transformer.h.{layer}."
        return {
            "ln1_w": sd[p + "ln_1.weight"], "ln1_b": sd[p + "ln_1.bias"],
            "wqkv": sd[p + "attn.c_attn.weight"].t().contiguous(), "bqkv": sd[p + "attn.c_attn.bias"],
            "wo": sd[p + "attn.c_proj.weight"].t().contiguous(), "bo": sd[p + "attn.c_proj.bias"],
            "ln2_w": sd[p + "ln_2.weight"], "ln2_b": sd[p + "ln_2.bias"],
            "w_fc": sd[p + "mlp.c_fc.weight"].t().contiguous(), "b_fc": sd[p + "mlp.c_fc.bias"],
            "w_proj": sd[p + "mlp.c_proj.weight"].t().contiguous(), "b_proj": sd[p + "mlp.c_proj.bias"],
        }
    p = f"model.layers.{layer}."
    out = {
        "attn_norm": sd[p + "input_layernorm.weight"],
        "wqkv": torch.cat([sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"],
                           sd[p + "self_attn.v_proj.weight"]], 0),
        "wo": sd[p + "self_attn.o_proj.weight"],
        "mlp_norm": sd[p + "post_attention_layernorm.weight"],
    }
    if cfg.is_moe and (p + "mlp.experts.gate_up_proj") in sd:
        # transformers>=5 in-memory layout: already fused [E, 2I, H] / [E, H, I]
        out["router"] = sd[p + "mlp.gate.weight"]
        out["experts_gate_up"] = sd[p + "mlp.experts.gate_up_proj"]
        out["experts_down"] = sd[p + "mlp.experts.down_proj"]
    elif cfg.is_moe:
        out["router"] = sd[p + "block_sparse_moe.gate.weight"]
        q = p + "block_sparse_moe.experts.{}."
        out["experts_gate_up"] = torch.stack([
            torch.cat([sd[q.format(e) + "w1.weight"], sd[q.format(e) + "w3.weight"]], 0)
            for e in range(cfg.num_experts)])
        out["experts_down"] = torch.stack([sd[q.format(e) + "w2.weight"] for e in range(cfg.num_experts)])
    else:
        out["w_gate_up"] = torch.cat([sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"]], 0)
        out["w_down"] = sd[p + "mlp.down_proj.weight"]
    return out


def hf_embed_names(cfg: ModelConfig) -> Dict[str, str]:
    if cfg.arch == "gpt2":
        return {"embed": "transformer.wte.weight", "pos_embed": "transformer.wpe.weight"}
    return {"embed": "model.embed_tokens.weight"}


def hf_head_names(cfg: ModelConfig) -> Dict[str, str]:
    if cfg.arch == "gpt2":
        return {"final_norm": "transformer.ln_f.weight", "final_norm_b": "transformer.ln_f.bias"}
    d = {"final_norm": "model.norm.weight"}
    if not cfg.tie_embeddings:
        d["lm_head"] = "lm_head.weight"
    return d


_LAYER_RE = re.compile(r"(?:^|\.)(?:layers|h|blocks|layer)\.(\d+)\.")


def layer_of(key: str) -> Optional[int]:
    """Block index of an HF parameter name (``model.layers.N.``, ``transformer.h.N.``,
    ``model.decoder.layers.N.``), or None for embeddings / final norm / head."""
    m = _LAYER_RE.search(key)
    return int(m.group(1)) if m else None


def is_embed_key(key: str) -> bool:
    return any(s in key for s in ("embed_tokens", "wte", "wpe", "embed_positions"))


def synth_block(cfg: ModelConfig, layer: int, seed: int, dtype, device) -> Dict[str, torch.Tensor]:
    return {n: synth_tensor(seed, layer, n, s, dtype, device) for n, s in block_shapes(cfg).items()}


def synth_embed(cfg: ModelConfig, seed: int, dtype, device) -> Dict[str, torch.Tensor]:
    return {n: synth_tensor(seed, EMBED, n, s, dtype, device) for n, s in embed_shapes(cfg).items()}


def synth_head(cfg: ModelConfig, seed: int, dtype, device) -> Dict[str, torch.Tensor]:
    return {n: synth_tensor(seed, HEAD, n, s, dtype, device) for n, s in head_shapes(cfg).items()}


def synth_hf_state_dict(cfg: ModelConfig, seed: int = 0, dtype=torch.float32,
                        layers: Optional[Iterable[int]] = None) -> Dict[str, torch.Tensor]:
    """A full HF-named random-init state dict (CPU), for writing test checkpoints."""
    sd: Dict[str, torch.Tensor] = {}
    e = synth_embed(cfg, seed, dtype, "cpu")
    for k, n in hf_embed_names(cfg).items():
        sd[n] = e[k]
    for layer in (layers if layers is not None else range(cfg.num_layers)):
        sd.update(block_to_hf(cfg, layer, synth_block(cfg, layer, seed, dtype, "cpu")))
    hd = synth_head(cfg, seed, dtype, "cpu")
    for k, n in hf_head_names(cfg).items():
        sd[n] = hd[k]
    if cfg.tie_embeddings and cfg.arch != "gpt2":
        pass
    if cfg.arch == "gpt2":
        sd["lm_head.weight"] = sd["transformer.wte.weight"]
    return sd
