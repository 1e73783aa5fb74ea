"""Pipeline schedule on ONE GPU: N stage threads (own HIP stream + decode graphs each) over the
loopback transport must reproduce the single-stage engine token for token."""
import pytest
import torch

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.models.stage import ModelStage
from distributed_llms_amd.parallel.pipeline import run_loopback_pipeline

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("stages", [2, 4])
def test_loopback_pipeline_gpu(cuda, stages):
    name = "tiny-llama-d128"
    cfg = get_model_config(name)
    sd = W.synth_hf_state_dict(cfg, seed=9, dtype=torch.float32)
    ecfg = EngineConfig(model=name, dtype="bfloat16", device="cuda", max_batch=4, max_seq_len=256,
                        num_kv_blocks=128, graph_batch_sizes=(1, 2, 4))
    prompts = [[i + 1, 2 * i + 3, 5, 7, 11 + i] for i in range(10)]
    p = SamplingParams(max_new_tokens=12, ignore_eos=True)
    ref = LLMEngine(ecfg, ModelStage(cfg, 0, cfg.num_layers, "cuda", torch.bfloat16).load_hf_state(sd)).generate(prompts, p)
    outs, drv, plan = run_loopback_pipeline(ecfg, stages, prompts, p, device="cuda", hf_state=sd)
    assert outs == ref
    assert drv.num_steps > 0
