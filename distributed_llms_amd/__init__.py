"""distributed_llms_amd: MI355X-native master/worker distributed LLM inference engine.

Same capabilities as MihirPanpatil/Distributed-LLMs (master/worker registration,
layer sharding, shard load/unload, request queue -> inference -> result), re-designed
for AMD Instinct MI355X (gfx950/CDNA4): contiguous layer slices resident in HBM,
hand-written HIP kernels on MFMA, RCCL point-to-point pipeline over xGMI.
"""
__version__ = "0.1.0"

from .config import EngineConfig, ModelConfig, PRESETS, get_model_config  # noqa: F401
