"""Model loading / downloading (API parity with ``src/model/loader.py`` and ``downloader.py``).

* :func:`download_model` -- the reference calls ``huggingface_hub.snapshot_download``
  (``src/model/downloader.py:4-6``).  This environment has no network, so the call is
  made with ``local_files_only=True`` (resolves the local HF cache) unless ``allow_network``.
* :func:`load_model` -- the reference loads a full ``transformers`` model on the master just
  to get its tokenizer (D14).  Here it returns ``(ModelStage, tokenizer_or_None)``: the
  stage holds every layer on ``device`` (a complete, runnable model in the engine's own
  layout); the tokenizer is loaded only if one exists locally.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple


def download_model(model_id: str, cache_dir: str = "./models", allow_network: bool = False) -> str:
    if os.path.isdir(model_id):
        return model_id
    from huggingface_hub import snapshot_download
    return snapshot_download(repo_id=model_id, cache_dir=cache_dir, local_files_only=not allow_network)


def load_tokenizer(model_path: str):
    try:
        from transformers import AutoTokenizer
        return AutoTokenizer.from_pretrained(model_path, local_files_only=True)
    except Exception:
        return None


def load_model(model_id: str, device_map: str = "auto", dtype: Optional[str] = None) -> Tuple[object, object]:
    """Load a checkpoint dir (HF layout or ``shards/``) or a ``synthetic:<preset>`` into one stage."""
    from ..config import get_model_config, resolve_device, torch_dtype
    from ..models.stage import ModelStage
    from .shard_manager import iter_checkpoint

    dev = resolve_device("auto" if device_map in (None, "auto") else device_map)
    dt = torch_dtype(dtype or ("bfloat16" if dev.startswith("cuda") else "float32"))
    cfg = get_model_config(model_id)
    stage = ModelStage(cfg, 0, cfg.num_layers, device=dev, dtype=dt)
    if model_id.startswith("synthetic:") or not os.path.isdir(model_id):
        stage.init_synthetic(0)
        return stage, None
    sd = dict(iter_checkpoint(model_id))
    if cfg.arch == "gpt2" and "lm_head.weight" in sd:
        sd.pop("lm_head.weight")
    stage.load_hf_state(sd)
    return stage, load_tokenizer(model_id)
