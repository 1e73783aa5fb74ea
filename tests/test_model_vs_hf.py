"""Golden numerics: our stage forward + greedy loop vs HF ``transformers`` on CPU.

The reference delegates modelling to ``transformers`` (``src/model/loader.py:5-25``);
here the same random-init HF-named state dict is loaded into both, and greedy
decodes must agree token for token (Llama-3 RoPE scaling, GQA, Mixtral top-2 MoE,
GPT-2 LayerNorm/GELU/learned positions, tied heads).
"""
import pytest
import torch
import transformers

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.models.stage import ModelStage


def _hf_model(cfg, sd):
    hfc = {k: v for k, v in cfg.to_hf_config().items()
           if not k.startswith("_") and k not in ("architectures", "model_type")}
    if cfg.arch == "gpt2":
        m = transformers.GPT2LMHeadModel(transformers.GPT2Config(**hfc))
        m.load_state_dict(sd, strict=False)
    elif cfg.arch == "mixtral":
        m = transformers.MixtralForCausalLM(transformers.MixtralConfig(**hfc))
        hsd = dict(sd)
        for l in range(cfg.num_layers):
            blk = W.hf_to_block(cfg, l, sd)
            p = f"model.layers.{l}."
            hsd[p + "mlp.gate.weight"] = blk["router"]
            hsd[p + "mlp.experts.gate_up_proj"] = blk["experts_gate_up"]
            hsd[p + "mlp.experts.down_proj"] = blk["experts_down"]
        missing, _ = m.load_state_dict(hsd, strict=False)
        assert not missing, missing
    else:
        m = transformers.LlamaForCausalLM(transformers.LlamaConfig(**hfc))
        missing, _ = m.load_state_dict(sd, strict=False)
        assert not missing, missing
    return m.eval()


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral", "tiny-gpt2"])
def test_greedy_matches_transformers(name):
    cfg = get_model_config(name)
    sd = W.synth_hf_state_dict(cfg, seed=3, dtype=torch.float32)
    m = _hf_model(cfg, sd)
    ecfg = EngineConfig(model=name, dtype="float32", device="cpu", max_batch=8, max_seq_len=256,
                        use_graphs=False, seed=3)
    stage = ModelStage(cfg, 0, cfg.num_layers, "cpu", torch.float32).load_hf_state(sd)
    eng = LLMEngine(ecfg, stage)
    prompts = [[5, 17, 33, 9, 100], [7, 8, 9, 10, 11, 12, 13, 40], [3]]
    outs = eng.generate(prompts, SamplingParams(max_new_tokens=10, ignore_eos=True))
    for p, o in zip(prompts, outs):
        with torch.no_grad():
            g = m.generate(torch.tensor([p]), max_new_tokens=10, min_new_tokens=10, do_sample=False,
                           pad_token_id=0)
        assert g[0, len(p):].tolist() == o


def test_prefill_logits_match_transformers():
    cfg = get_model_config("tiny-llama")
    sd = W.synth_hf_state_dict(cfg, seed=11, dtype=torch.float32)
    m = _hf_model(cfg, sd)
    ecfg = EngineConfig(model="tiny-llama", dtype="float32", device="cpu", max_batch=4, max_seq_len=128,
                        use_graphs=False)
    stage = ModelStage(cfg, 0, cfg.num_layers, "cpu", torch.float32).load_hf_state(sd)
    eng = LLMEngine(ecfg, stage)
    prompt = [1, 50, 60, 70, 80, 90]
    seq = eng.add_request(prompt, SamplingParams(max_new_tokens=1))
    from distributed_llms_amd.engine.batch import build_host_batch
    st = eng.scheduler.schedule(0)
    hb = build_host_batch(st, eng.bm, 32)
    logits = eng.runner.execute(hb)
    with torch.no_grad():
        ref = m(torch.tensor([prompt])).logits[0, -1]
    torch.testing.assert_close(logits[0], ref, atol=1e-4, rtol=1e-4)
