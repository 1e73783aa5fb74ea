"""Debug: determinism of a 3-stage sub-layer plan ((0,8),(8,11),(11,20), group 5) on one GPU."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.models.stage import ModelStage
from distributed_llms_amd.parallel import pipeline as P
from distributed_llms_amd.parallel import planner

name = "tiny-llama-d128"
cfg = get_model_config(name)
sd = W.synth_hf_state_dict(cfg, seed=3, dtype=torch.float32)
units = [tuple(int(x) for x in u.split(",")) for u in (sys.argv[1] if len(sys.argv) > 1 else "0,8;8,11;11,20").split(";")]
forced = planner.StagePlan(tuple((a // 5, (b + 4) // 5) for a, b in units), tuple(0.0 for _ in units), tuple(units), 5)
P.plan_units = lambda *a, **k: forced            # run_loopback_pipeline imports it at call time
planner.plan_units = lambda *a, **k: forced
prompts = [[i + 1, 2 * i + 3, 5, 7, 11 + i] for i in range(10)]
p = SamplingParams(max_new_tokens=12, ignore_eos=True)
for graphs in (True, False):
    ecfg = EngineConfig(model=name, dtype="bfloat16", device="cuda", max_batch=4, max_seq_len=256,
                        num_kv_blocks=128, graph_batch_sizes=(1, 2, 4), use_graphs=graphs)
    ref = LLMEngine(ecfg, ModelStage(cfg, 0, cfg.num_layers, "cuda", torch.bfloat16).load_hf_state(sd)).generate(prompts, p)
    for r in range(3):
        outs, drv, plan = P.run_loopback_pipeline(ecfg, len(units), prompts, p, device="cuda", hf_state=sd)
        print(f"graphs={graphs} round {r}: plan {plan.units} agree {sum(o == q for o, q in zip(outs, ref))}/10",
              [i for i, (o, q) in enumerate(zip(outs, ref)) if o != q], flush=True)
