"""Model presets and engine configuration.

The reference hard-codes every knob as a constructor default or literal
(``src/master/node.py:15``, ``src/worker/node.py:35,52-65``, ``run_master.py:17``;
SURVEY §2.7) and its docs promise a YAML/JSON config system that was never
written (``plan.md:70-73``).  Here there is one :class:`EngineConfig` dataclass,
loadable from JSON/YAML and overridable from CLI flags, plus :class:`ModelConfig`
presets for the model families named in ``BASELINE.json``.

Model dimensions are the public HF ``config.json`` values, not
reference data.
"""
from __future__ import annotations

import dataclasses
import json
import os
from dataclasses import dataclass, field
from typing import Any, Dict, Optional


@dataclass
class ModelConfig:
    name: str
    arch: str                      # "llama" (Llama-2/3), "mixtral", "gpt2"
    vocab_size: int
    hidden_size: int
    intermediate_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    max_position: int = 8192
    rope_theta: float = 10000.0
    rope_scaling: Optional[Dict[str, Any]] = None
    norm_eps: float = 1e-5
    tie_embeddings: bool = False
    num_experts: int = 0           # MoE (Mixtral): experts per layer
    experts_per_token: int = 0     # MoE top-k
    bos_token_id: int = 1
    eos_token_id: int = 2

    # ------------------------------------------------------------------ sizes
    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    def layer_param_count(self) -> int:
        h, i = self.hidden_size, self.intermediate_size
        attn = h * self.qkv_size + self.q_size * h
        if self.arch == "gpt2":
            attn += self.qkv_size + h  # biases
            mlp = 2 * h * i + i + h
            norms = 4 * h
        elif self.is_moe:
            mlp = self.num_experts * 3 * h * i + self.num_experts * h
            norms = 2 * h
        else:
            mlp = 3 * h * i
            norms = 2 * h
        return attn + mlp + norms

    def embed_param_count(self) -> int:
        n = self.vocab_size * self.hidden_size
        if self.arch == "gpt2":
            n += self.max_position * self.hidden_size
        return n

    def head_param_count(self) -> int:
        """Final norm + LM head (0 extra for tied heads other than the norm)."""
        norm = self.hidden_size * (2 if self.arch == "gpt2" else 1)
        return norm + (0 if self.tie_embeddings else self.vocab_size * self.hidden_size)

    def param_count(self) -> int:
        return (self.embed_param_count() + self.num_layers * self.layer_param_count()
                + self.head_param_count())

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    # ----------------------------------------------------------- HF interop
    def to_hf_config(self) -> Dict[str, Any]:
        """A ``config.json``-compatible dict (written into ``shards/config.json``)."""
        if self.arch == "gpt2":
            return {
                "model_type": "gpt2", "architectures": ["GPT2LMHeadModel"],
                "vocab_size": self.vocab_size, "n_embd": self.hidden_size,
                "n_layer": self.num_layers, "n_head": self.num_heads,
                "n_inner": self.intermediate_size, "n_positions": self.max_position,
                "layer_norm_epsilon": self.norm_eps, "tie_word_embeddings": True,
                "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
                "activation_function": "gelu_new", "_dllm_name": self.name,
            }
        d = {
            "model_type": "mixtral" if self.is_moe else "llama",
            "architectures": ["MixtralForCausalLM" if self.is_moe else "LlamaForCausalLM"],
            "vocab_size": self.vocab_size, "hidden_size": self.hidden_size,
            "intermediate_size": self.intermediate_size,
            "num_hidden_layers": self.num_layers, "num_attention_heads": self.num_heads,
            "num_key_value_heads": self.num_kv_heads, "head_dim": self.head_dim,
            "max_position_embeddings": self.max_position, "rope_theta": self.rope_theta,
            "rms_norm_eps": self.norm_eps, "tie_word_embeddings": self.tie_embeddings,
            "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
            "hidden_act": "silu", "_dllm_name": self.name,
        }
        if self.rope_scaling:
            d["rope_scaling"] = dict(self.rope_scaling)
        if self.is_moe:
            d["num_local_experts"] = self.num_experts
            d["num_experts_per_tok"] = self.experts_per_token
        return d

    @staticmethod
    def from_hf_config(cfg: Dict[str, Any], name: Optional[str] = None) -> "ModelConfig":
        mt = cfg.get("model_type", "llama")
        name = name or cfg.get("_dllm_name") or cfg.get("_name_or_path") or mt
        eos = cfg.get("eos_token_id", 2)
        if isinstance(eos, list):
            eos = eos[0]
        if mt == "gpt2":
            h = cfg["n_embd"]
            return ModelConfig(
                name=name, arch="gpt2", vocab_size=cfg["vocab_size"], hidden_size=h,
                intermediate_size=cfg.get("n_inner") or 4 * h, num_layers=cfg["n_layer"],
                num_heads=cfg["n_head"], num_kv_heads=cfg["n_head"],
                head_dim=h // cfg["n_head"], max_position=cfg.get("n_positions", 1024),
                norm_eps=cfg.get("layer_norm_epsilon", 1e-5), tie_embeddings=True,
                bos_token_id=cfg.get("bos_token_id", 50256), eos_token_id=eos)
        if mt not in ("llama", "mixtral", "mistral"):
            raise ValueError(f"unsupported model_type {mt!r} (supported: llama, mistral, mixtral, gpt2)")
        h = cfg["hidden_size"]
        nh = cfg["num_attention_heads"]
        return ModelConfig(
            name=name, arch="mixtral" if mt == "mixtral" else "llama",
            vocab_size=cfg["vocab_size"], hidden_size=h,
            intermediate_size=cfg["intermediate_size"], num_layers=cfg["num_hidden_layers"],
            num_heads=nh, num_kv_heads=cfg.get("num_key_value_heads", nh),
            head_dim=cfg.get("head_dim") or h // nh,
            max_position=cfg.get("max_position_embeddings", 4096),
            rope_theta=cfg.get("rope_theta", 10000.0), rope_scaling=cfg.get("rope_scaling"),
            norm_eps=cfg.get("rms_norm_eps", 1e-5),
            tie_embeddings=bool(cfg.get("tie_word_embeddings", False)),
            num_experts=cfg.get("num_local_experts", 0) if mt == "mixtral" else 0,
            experts_per_token=cfg.get("num_experts_per_tok", 0) if mt == "mixtral" else 0,
            bos_token_id=cfg.get("bos_token_id", 1), eos_token_id=eos)


_LLAMA3_ROPE = {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0,
                "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}

PRESETS: Dict[str, ModelConfig] = {
    "llama3-8b": ModelConfig(
        name="llama3-8b", arch="llama", vocab_size=128256, hidden_size=4096,
        intermediate_size=14336, num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128,
        max_position=8192, rope_theta=500000.0, rope_scaling=dict(_LLAMA3_ROPE),
        norm_eps=1e-5, bos_token_id=128000, eos_token_id=128001),
    "llama3-70b": ModelConfig(
        name="llama3-70b", arch="llama", vocab_size=128256, hidden_size=8192,
        intermediate_size=28672, num_layers=80, num_heads=64, num_kv_heads=8, head_dim=128,
        max_position=8192, rope_theta=500000.0, rope_scaling=dict(_LLAMA3_ROPE),
        norm_eps=1e-5, bos_token_id=128000, eos_token_id=128001),
    "mixtral-8x7b": ModelConfig(
        name="mixtral-8x7b", arch="mixtral", vocab_size=32000, hidden_size=4096,
        intermediate_size=14336, num_layers=32, num_heads=32, num_kv_heads=8, head_dim=128,
        max_position=32768, rope_theta=1000000.0, norm_eps=1e-5,
        num_experts=8, experts_per_token=2, bos_token_id=1, eos_token_id=2),
    "gpt2-small": ModelConfig(
        name="gpt2-small", arch="gpt2", vocab_size=50257, hidden_size=768,
        intermediate_size=3072, num_layers=12, num_heads=12, num_kv_heads=12, head_dim=64,
        max_position=1024, norm_eps=1e-5, tie_embeddings=True,
        bos_token_id=50256, eos_token_id=50256),
    # Tiny configs with the same structure, for CPU tests and GPU smoke runs.
    "tiny-llama": ModelConfig(
        name="tiny-llama", arch="llama", vocab_size=512, hidden_size=256,
        intermediate_size=512, num_layers=4, num_heads=4, num_kv_heads=2, head_dim=64,
        max_position=1024, rope_theta=500000.0, rope_scaling=dict(_LLAMA3_ROPE, original_max_position_embeddings=256),
        norm_eps=1e-5, bos_token_id=1, eos_token_id=2),
    "tiny-llama-d128": ModelConfig(
        name="tiny-llama-d128", arch="llama", vocab_size=1024, hidden_size=512,
        intermediate_size=1024, num_layers=4, num_heads=4, num_kv_heads=1, head_dim=128,
        max_position=2048, rope_theta=500000.0, norm_eps=1e-5, bos_token_id=1, eos_token_id=2),
    "tiny-mixtral": ModelConfig(
        name="tiny-mixtral", arch="mixtral", vocab_size=512, hidden_size=256,
        intermediate_size=384, num_layers=4, num_heads=4, num_kv_heads=2, head_dim=64,
        max_position=1024, rope_theta=1000000.0, norm_eps=1e-5,
        num_experts=4, experts_per_token=2, bos_token_id=1, eos_token_id=2),
    "tiny-gpt2": ModelConfig(
        name="tiny-gpt2", arch="gpt2", vocab_size=512, hidden_size=128,
        intermediate_size=512, num_layers=4, num_heads=2, num_kv_heads=2, head_dim=64,
        max_position=512, norm_eps=1e-5, tie_embeddings=True, bos_token_id=0, eos_token_id=0),
}


def get_model_config(spec: str) -> ModelConfig:
    """Resolve ``spec``: a preset name, ``synthetic:<preset>``, or a directory with ``config.json``.
    ``<preset>@<N>l``: the preset's dimensions with N layers (full-size layer shapes at a depth a
    test or a one-GPU rehearsal can afford, e.g. ``llama3-70b@4l``)."""
    if spec.startswith("synthetic:"):
        spec = spec.split(":", 1)[1]
    if "@" in spec and spec.rsplit("@", 1)[0] in PRESETS:
        base, depth = spec.rsplit("@", 1)
        if not (depth.endswith("l") and depth[:-1].isdigit() and int(depth[:-1]) >= 1):
            raise KeyError(f"model {spec!r}: expected <preset>@<layers>l, e.g. {base}@4l")
        return dataclasses.replace(PRESETS[base], name=spec, num_layers=int(depth[:-1]))
    if spec in PRESETS:
        return dataclasses.replace(PRESETS[spec])
    for cand in (os.path.join(spec, "config.json"), os.path.join(spec, "shards", "config.json"), spec):
        if os.path.isfile(cand) and cand.endswith(".json"):
            with open(cand) as f:
                return ModelConfig.from_hf_config(json.load(f))
    raise KeyError(f"unknown model {spec!r}; presets: {sorted(PRESETS)}")


@dataclass
class EngineConfig:
    """Everything the master decides; workers receive their slice in the REGISTER reply."""
    model: str = "synthetic:llama3-8b"
    dtype: str = "bfloat16"
    device: str = "auto"               # "auto" -> cuda if available else cpu
    num_workers: int = 1               # pipeline stages (one process / GPU each)
    dp_replicas: int = 1               # data-parallel replica groups (dp x pp = world)
    microbatches: int = 0              # 0 -> pipeline_slots(): stages + 1 on GPUs, stages on CPUs
    # single-GPU engine: microbatch slots interleaved on HIP streams.  1 by default: decode GEMMs
    # are weight-streaming, and two half-batches stream every weight twice (measured 16.2k vs
    # 21.0k tok/s at batch 256, profiles/dual_stream.txt)
    streams: int = 1
    max_batch: int = 256               # max sequences decoded per step (per replica)
    max_prefill_tokens: int = 16384    # max prompt tokens per prefill step
    # prompt tokens a step may add to a slot's running decode rows (mixed prefill + decode step,
    # SURVEY §5.7; capped by max_prefill_tokens): arrivals during decode are prefilled in chunks
    # riding along with the decode batch instead of prefill-only steps that stall every running
    # sequence; 0 = prefill-first (a step is all prefill or all decode).  The budget trades the
    # running rows' inter-token latency against admission speed: a 512-token budget made the
    # pipeline's burst admission (256 prompts per slot behind 64 decode rows) take 48 small eager
    # steps instead of 3 full ones (pp2 rehearsal 17.4k vs 27k tok/s), so the default admits at
    # the full prefill rate and latency-bound deployments lower it (profiles/round5_open_loop.md)
    mixed_prefill_tokens: int = 8192
    max_seq_len: int = 4096
    kv_block_size: int = 32            # tokens per paged-KV block
    kv_cache_fraction: float = 0.80    # of free HBM after weights
    num_kv_blocks: int = 0             # 0 -> derive from kv_cache_fraction
    use_graphs: bool = True            # HIP-graph capture of the decode step
    quant: str = "none"                # "fp8": W8A8 e4m3 dense projections (ops/quant.py)
    # pipeline activation transport between GPU stages: "auto" (= "rccl" on GPUs), "rccl" (native
    # RCCL p2p, one communicator per edge, static rings), "torch" (torch.distributed's RCCL group),
    # "ipc" (HIP-IPC peer writes); CPU stages always use torch.distributed (gloo)
    transport: str = "auto"
    comm_timeout_s: float = 600.0      # a pipeline peer silent this long -> the rank raises (no hang)
    graph_batch_sizes: tuple = (1, 2, 4, 8, 16, 32, 48, 64, 96, 128, 192, 256)
    # kernel-dispatch overrides ({knob: value}, distributed_llms_amd/knobs.py), applied when a stage
    # runner is built; empty = the measured defaults
    kernel_knobs: Dict[str, Any] = field(default_factory=dict)
    host: str = "0.0.0.0"
    port: int = 65432
    worker_port: int = 65433
    heartbeat_interval: float = 5.0
    heartbeat_timeout: float = 20.0
    request_timeout: float = 600.0
    seed: int = 0
    shard_dir: Optional[str] = None    # checkpoint dir (shards/); None -> synthetic init
    log_level: str = "INFO"

    def validate(self) -> None:
        if self.dtype not in ("bfloat16", "float16", "float32"):
            raise ValueError(f"dtype {self.dtype}")
        if self.num_workers < 1 or self.dp_replicas < 1:
            raise ValueError("num_workers and dp_replicas must be >= 1")
        if self.kv_block_size not in (16, 32, 64):
            raise ValueError("kv_block_size must be 16, 32 or 64")
        if self.quant not in ("none", "fp8"):
            raise ValueError(f"quant {self.quant!r} (none, fp8)")
        if self.transport not in ("auto", "rccl", "torch", "ipc"):
            raise ValueError(f"transport {self.transport!r} (auto, rccl, torch, ipc)")
        if self.comm_timeout_s <= 0:
            raise ValueError("comm_timeout_s must be > 0")
        from . import knobs
        unknown = set(self.kernel_knobs) - set(knobs.as_dict())
        if unknown:
            raise ValueError(f"unknown kernel_knobs {sorted(unknown)}")
        if self.max_batch < 1 or self.max_seq_len < 2:
            raise ValueError("max_batch/max_seq_len")
        cfg = get_model_config(self.model if self.shard_dir is None else self.shard_dir)
        if self.num_workers > cfg.num_layers:
            raise ValueError(f"{self.num_workers} stages > {cfg.num_layers} layers")

    def model_config(self) -> ModelConfig:
        return get_model_config(self.shard_dir or self.model)

    def to_dict(self) -> Dict[str, Any]:
        d = dataclasses.asdict(self)
        d["graph_batch_sizes"] = list(self.graph_batch_sizes)
        return d

    @staticmethod
    def from_dict(d: Dict[str, Any]) -> "EngineConfig":
        names = {f.name for f in dataclasses.fields(EngineConfig)}
        unknown = set(d) - names
        if unknown:
            raise ValueError(f"unknown config keys: {sorted(unknown)}")
        d = dict(d)
        if "graph_batch_sizes" in d:
            d["graph_batch_sizes"] = tuple(d["graph_batch_sizes"])
        return EngineConfig(**d)

    @staticmethod
    def from_file(path: str) -> "EngineConfig":
        with open(path) as f:
            if path.endswith((".yaml", ".yml")):
                import yaml
                data = yaml.safe_load(f) or {}
            else:
                data = json.load(f)
        return EngineConfig.from_dict(data)

    def apply_overrides(self, **kw) -> "EngineConfig":
        kw = {k: v for k, v in kw.items() if v is not None}
        return dataclasses.replace(self, **kw)


def pipeline_slots(ecfg: "EngineConfig", pp: int, device=None) -> int:
    """Microbatch slots of a pp-stage pipeline (``ecfg.microbatches`` when set).

    GPU stages: pp + 1 -- one per stage keeps every stage busy only if the ring closure (sampled
    ids back to stage 0) were free; the spare slot covers the hops.  CPU stages: pp -- a CPU
    stage at these batch sizes is bound by streaming its weights, which every extra microbatch
    re-reads (GPT-2 small on two 4-core stages: 140 tok/s with 3 slots, 184 with 2), while its
    hops are cheap next to a step.  ``device`` is the stages' device (``ecfg.device`` if None).
    """
    if ecfg.microbatches > 0:
        return ecfg.microbatches
    if pp <= 1:
        return 1
    dev = str(device if device is not None else ecfg.device)
    if dev == "auto":
        dev = resolve_device(dev)
    return pp if dev.startswith("cpu") else pp + 1


def resolve_device(spec: str = "auto") -> str:
    import torch
    if spec == "auto":
        return "cuda" if torch.cuda.is_available() else "cpu"
    return spec


def torch_dtype(name: str):
    import torch
    return {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}[name]
