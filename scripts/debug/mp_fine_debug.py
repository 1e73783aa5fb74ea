"""Debug: multi-process GPU pipeline (stage processes on one GPU) with forced unit plans."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_pipeline_gpu import _mp_ecfg, _run_ranks   # noqa: E402
from distributed_llms_amd.engine.llm_engine import LLMEngine   # noqa: E402
from distributed_llms_amd.engine.sequence import SamplingParams   # noqa: E402

if __name__ == "__main__":
    prompts = [[i + 1, 2 * i + 3, 5, 7, 11 + i] for i in range(10)]
    ref = LLMEngine(_mp_ecfg(1)).generate(prompts, SamplingParams(max_new_tokens=12, ignore_eos=True))
    for spec in sys.argv[2:]:
        os.environ["DLLM_PP_UNITS"] = spec
        world = spec.count(";") + 1
        out = _run_ranks(world, prompts, sys.argv[1], rounds=3, fine="1")[0]
        print(f"{sys.argv[1] or 'gloo'} {spec}: " + "  ".join(
            f"r{r} agree {sum(o == q for o, q in zip(rr, ref))}/10 {[i for i, (o, q) in enumerate(zip(rr, ref)) if o != q]}"
            for r, rr in enumerate(out)), flush=True)
