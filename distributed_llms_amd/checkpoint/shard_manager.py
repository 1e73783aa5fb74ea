"""Checkpoint sharding into the reference's on-disk layout, made pipeline-correct.

Layout kept from the reference (``src/model/shard_manager.py:11,64-74``):
  <model_path>/shards/shard_{i}.pt        torch.save'd {hf_param_name: tensor}
  <model_path>/shards/shard_info.json     {"<i>": [hf_param_names...]}
  <model_path>/shards/config.json         copy of the HF config
Additive extension (ignored by reference readers):
  <model_path>/shards/shard_plan.json     {"ranges": [[a, b), ...], "embed_shard": 0, "head_shard": n-1,
                                           "sha256": {...}, "bytes": [...]}
  <model_path>/shards/shard_{i}.safetensors  (optional twin for zero-copy mmap loads)

Fixed defects of the reference: keys are grouped by their real block index for every
HF naming scheme (``model.layers.N.``, ``transformer.h.N.``, ``model.decoder.layers.N.``;
D11 kept only ``key.split('.')[1]`` digits); each shard is ONE contiguous, cost-balanced
layer range (D12 interleaved them); embeddings go to shard 0 and final norm / LM head to
the last shard (D11 dropped them); single-file ``model.safetensors`` and multi-file
``model-0000x-of-0000y.safetensors`` + index checkpoints are read with safetensors (D13
fed safetensors to torch.load); ``.bin`` checkpoints load with ``weights_only=True``.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch

from ..config import ModelConfig
from ..models import weights as W
from ..parallel.planner import StagePlan, plan_stages


# ----------------------------------------------------------------- readers
def checkpoint_files(model_path: str) -> List[str]:
    idx = os.path.join(model_path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            wm = json.load(f)["weight_map"]
        return sorted({os.path.join(model_path, v) for v in wm.values()})
    for name in ("model.safetensors", "pytorch_model.bin"):
        p = os.path.join(model_path, name)
        if os.path.exists(p):
            return [p]
    multi = sorted(glob.glob(os.path.join(model_path, "pytorch_model-*.bin")))
    if multi:
        return multi
    raise FileNotFoundError(f"no checkpoint (model.safetensors[.index.json] / pytorch_model.bin) in {model_path}")


def _load_bin(path: str) -> Dict[str, torch.Tensor]:
    """A ``.bin`` checkpoint, memory-mapped where the file is a zip archive (tensors are paged in
    when touched, never unpickled objects: weights_only)."""
    try:
        return torch.load(path, map_location="cpu", weights_only=True, mmap=True)
    except RuntimeError:            # legacy (non-zip) torch.save format cannot be mmapped
        return torch.load(path, map_location="cpu", weights_only=True)


def iter_checkpoint(model_path: str, keys: Optional[set] = None) -> Iterable[Tuple[str, torch.Tensor]]:
    """Yield (name, tensor); safetensors files are read lazily, key by key, and ``.bin`` files
    memory-mapped -- a file whose keys are all outside ``keys`` is not read at all."""
    for f in checkpoint_files(model_path):
        if f.endswith(".safetensors"):
            from safetensors import safe_open
            with safe_open(f, framework="pt") as sf:
                for k in sf.keys():
                    if keys is None or k in keys:
                        yield k, sf.get_tensor(k)
        else:
            sd = _load_bin(f)
            for k, v in sd.items():
                if keys is None or k in keys:
                    yield k, v
            del sd


def checkpoint_index(model_path: str) -> Dict[str, Tuple[str, int]]:
    """name -> (file, bytes) without materialising any tensor (safetensors headers; mmapped .bin)."""
    out: Dict[str, Tuple[str, int]] = {}
    for f in checkpoint_files(model_path):
        if f.endswith(".safetensors"):
            from safetensors import safe_open
            with safe_open(f, framework="pt") as sf:
                for k in sf.keys():
                    sl = sf.get_slice(k)
                    n = 1
                    for d in sl.get_shape():
                        n *= int(d)
                    out[k] = (f, n * _DTYPE_BYTES.get(sl.get_dtype(), 4))
        else:
            sd = _load_bin(f)
            for k, v in sd.items():
                out[k] = (f, v.numel() * v.element_size())
            del sd
    return out


_DTYPE_BYTES = {"F64": 8, "F32": 4, "F16": 2, "BF16": 2, "I64": 8, "I32": 4, "I16": 2, "I8": 1, "U8": 1,
                "BOOL": 1, "F8_E4M3": 1, "F8_E5M2": 1}


def checkpoint_keys(model_path: str) -> List[str]:
    return list(checkpoint_index(model_path))


def load_shard_file(path: str) -> Dict[str, torch.Tensor]:
    """Load one shard file without executing anything from it."""
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return torch.load(path, map_location="cpu", weights_only=True)


def load_shard_bytes(data: bytes) -> Dict[str, torch.Tensor]:
    """Shard bytes received over the wire: safetensors or a torch.save zip (weights only)."""
    import io
    if data[:4] == b"PK\x03\x04":        # torch.save zip archive
        return torch.load(io.BytesIO(data), map_location="cpu", weights_only=True)
    from safetensors.torch import load
    return load(data)


def _sha256(path: str) -> str:
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for chunk in iter(lambda: f.read(1 << 24), b""):
            h.update(chunk)
    return h.hexdigest()


def assign_key(key: str, plan: StagePlan, num_layers: int) -> int:
    layer = W.layer_of(key)
    if layer is not None:
        if layer >= num_layers:
            raise ValueError(f"{key}: layer {layer} >= num_layers {num_layers}")
        return plan.stage_of_layer(layer)
    if W.is_embed_key(key):
        return 0
    return plan.num_stages - 1          # final norm, lm_head, anything global


class ModelShardManager:
    def __init__(self, model_path: str, num_shards: int, config: Optional[ModelConfig] = None):
        self.model_path = model_path
        self.num_shards = num_shards
        self.shard_dir = os.path.join(model_path, "shards")
        self.shard_info: Dict[int, List[str]] = {}
        self.config = config
        self.plan: Optional[StagePlan] = None

    def _hf_config(self) -> dict:
        with open(os.path.join(self.model_path, "config.json")) as f:
            return json.load(f)

    def shard_model(self, write_safetensors: bool = False, checksums: bool = True) -> str:
        """Write ``shards/`` one shard at a time: the key -> stage assignment comes from the
        checkpoint index (no tensor read), then each shard's tensors are read (safetensors: per
        key; ``.bin``: memory-mapped), written and dropped before the next shard is read.  Peak host
        memory is about one shard -- a 141 GB Llama-3-70B checkpoint shards on a host with far less
        RAM (the reference's shard_model held the whole state dict, src/model/shard_manager.py:17-61)."""
        hf = self._hf_config()
        cfg = self.config or ModelConfig.from_hf_config(hf)
        n = min(self.num_shards, cfg.num_layers)
        if n != self.num_shards:
            raise ValueError(f"{self.num_shards} shards > {cfg.num_layers} layers")
        self.plan = plan_stages(cfg, n)
        os.makedirs(self.shard_dir, exist_ok=True)
        index = checkpoint_index(self.model_path)
        tied = cfg.tie_embeddings
        members: List[List[str]] = [[] for _ in range(n)]
        for k in index:
            if k == "lm_head.weight" and tied:
                continue          # tied head == embedding (GPT-2 style); the last stage re-uses it
            members[assign_key(k, self.plan, cfg.num_layers)].append(k)
        if tied and n > 1:
            emb = W.hf_embed_names(cfg)["embed"]
            if emb in index:
                members[-1].append(emb)
        sizes, sums = [], {}
        for i, keys in enumerate(members):
            want = set(keys)
            sd = {k: v for k, v in iter_checkpoint(self.model_path, want)}
            sd = {k: sd[k] for k in keys if k in sd}         # checkpoint order within the shard
            path = os.path.join(self.shard_dir, f"shard_{i}.pt")
            torch.save(sd, path)
            if write_safetensors:
                from safetensors.torch import save_file
                save_file({k: v.contiguous() for k, v in sd.items()},
                          os.path.join(self.shard_dir, f"shard_{i}.safetensors"))
            self.shard_info[i] = list(sd.keys())
            sizes.append(sum(t.numel() * t.element_size() for t in sd.values()))
            del sd
            if checksums:
                sums[f"shard_{i}.pt"] = _sha256(path)
        with open(os.path.join(self.shard_dir, "shard_info.json"), "w") as f:
            json.dump({str(k): v for k, v in self.shard_info.items()}, f)
        with open(os.path.join(self.shard_dir, "config.json"), "w") as f:
            json.dump(hf, f)
        with open(os.path.join(self.shard_dir, "shard_plan.json"), "w") as f:
            json.dump({"num_shards": n, "ranges": [list(r) for r in self.plan.ranges], "embed_shard": 0,
                       "head_shard": n - 1, "bytes": sizes, "sha256": sums, "model": cfg.name}, f, indent=1)
        return self.shard_dir

    def get_shard_paths(self) -> List[str]:
        return [os.path.join(self.shard_dir, f"shard_{i}.pt") for i in range(self.num_shards)]

    @staticmethod
    def read_plan(shard_dir: str) -> dict:
        with open(os.path.join(shard_dir, "shard_plan.json")) as f:
            return json.load(f)

    @staticmethod
    def verify(shard_dir: str) -> bool:
        """Re-hash the shard files against shard_plan.json."""
        plan = ModelShardManager.read_plan(shard_dir)
        return all(_sha256(os.path.join(shard_dir, f)) == h for f, h in plan.get("sha256", {}).items())

    @staticmethod
    def reconstruct_model(shard_paths, config_path) -> Tuple[Dict[str, torch.Tensor], dict]:
        with open(config_path) as f:
            config = json.load(f)
        full: Dict[str, torch.Tensor] = {}
        for p in shard_paths:
            full.update(load_shard_file(p))
        return full, config


def write_synthetic_checkpoint(preset: str, out_dir: str, seed: int = 0, dtype=torch.float32,
                               safetensors: bool = True) -> str:
    """A random-init HF-layout checkpoint (config.json + weights), for tests and demos (no network)."""
    from ..config import get_model_config
    cfg = get_model_config(preset)
    os.makedirs(out_dir, exist_ok=True)
    sd = W.synth_hf_state_dict(cfg, seed=seed, dtype=dtype)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(cfg.to_hf_config(), f, indent=1)
    if safetensors:
        from safetensors.torch import save_file
        if cfg.arch == "gpt2":
            sd = {k: v for k, v in sd.items() if k != "lm_head.weight"}
        save_file({k: v.contiguous() for k, v in sd.items()}, os.path.join(out_dir, "model.safetensors"))
    else:
        torch.save(sd, os.path.join(out_dir, "pytorch_model.bin"))
    return out_dir
