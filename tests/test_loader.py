"""Model loading / downloading and tokenization (the reference's ``src/model/loader.py``,
``downloader.py`` and its tests ``tests/model/test_loader.py``).

The reference's loader tests mock ``from_pretrained``; here the real functions run offline:
``download_model`` resolves local paths and a local Hugging Face cache snapshot (no network in
this environment: ``local_files_only`` unless ``allow_network``), ``load_model`` builds a complete
stage from a synthetic preset or an HF-layout directory, and the byte tokenizer round-trips."""
import json
import os

import pytest
import torch

from distributed_llms_amd.checkpoint.loader import download_model, load_model, load_tokenizer
from distributed_llms_amd.config import get_model_config
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.utils.tokenizer import ByteTokenizer, get_tokenizer


def test_download_model_returns_local_directories_unchanged(tmp_path):
    assert download_model(str(tmp_path)) == str(tmp_path)


def test_download_model_resolves_a_local_hf_cache_snapshot(tmp_path):
    """A snapshot already in the cache (``models--<org>--<name>/snapshots/<rev>``, ``refs/main``)
    is found without the network -- what the reference's snapshot_download call returns."""
    repo = tmp_path / "models--acme--tiny"
    snap = repo / "snapshots" / "0123abcd"
    snap.mkdir(parents=True)
    (snap / "config.json").write_text(json.dumps({"model_type": "llama"}))
    (repo / "refs").mkdir()
    (repo / "refs" / "main").write_text("0123abcd")
    path = download_model("acme/tiny", cache_dir=str(tmp_path))
    assert os.path.realpath(path) == os.path.realpath(str(snap))
    assert os.path.exists(os.path.join(path, "config.json"))


def test_download_model_without_network_fails_loudly(tmp_path):
    with pytest.raises(Exception):
        download_model("acme/not-cached", cache_dir=str(tmp_path))


def test_load_model_synthetic_preset_is_a_complete_stage():
    stage, tok = load_model("synthetic:tiny-llama", device_map="cpu")
    cfg = get_model_config("tiny-llama")
    assert tok is None
    assert stage.is_first and stage.is_last and len(stage.layers) == cfg.num_layers
    assert stage.weight_bytes() > 0 and stage.dtype == torch.float32


def test_load_model_reads_an_hf_layout_directory(tmp_path):
    """An HF directory (config.json + model.safetensors) loads into one stage whose tensors are the
    checkpoint's (q|k|v and gate|up fused in the engine's layout)."""
    from distributed_llms_amd.checkpoint.shard_manager import write_synthetic_checkpoint
    cfg = get_model_config("tiny-llama")
    write_synthetic_checkpoint("tiny-llama", str(tmp_path), seed=4)
    sd = W.synth_hf_state_dict(cfg, seed=4, dtype=torch.float32)
    stage, tok = load_model(str(tmp_path), device_map="cpu", dtype="float32")
    assert tok is None                                       # no tokenizer files in the directory
    ref = W.hf_to_block(cfg, 0, sd)
    for name, t in ref.items():
        torch.testing.assert_close(stage.layers[0][name], t)
    assert load_tokenizer(str(tmp_path)) is None


def test_byte_tokenizer_round_trips_utf8():
    tok = ByteTokenizer()
    text = "héllo, wörld — 8 GPUs"
    ids = tok.encode(text)
    assert all(3 <= i < 259 for i in ids)
    assert tok.decode(ids) == text
    assert tok.encode("") == [ByteTokenizer.OFFSET]          # never an empty prompt
    with pytest.raises(ValueError):
        ByteTokenizer(100)


def test_get_tokenizer_falls_back_to_bytes_and_wraps_hf():
    assert isinstance(get_tokenizer(None, vocab_size=128256), ByteTokenizer)

    class Fake:
        def __call__(self, text):
            return {"input_ids": [len(text), 7]}

        def decode(self, ids, skip_special_tokens=True):
            return "|".join(map(str, ids))

    t = get_tokenizer(Fake())
    assert t.encode("abc") == [3, 7] and t.decode([1, 2]) == "1|2"
