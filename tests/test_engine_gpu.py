"""End-to-end engine on the GPU: HIP kernel path vs the CPU fp32 reference path."""
import pytest
import torch

from distributed_llms_amd import _ext
from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.batch import build_host_batch
from distributed_llms_amd.engine.llm_engine import LLMEngine
from distributed_llms_amd.engine.sequence import SamplingParams
from distributed_llms_amd.models import weights as W
from distributed_llms_amd.models.stage import ModelStage

pytestmark = pytest.mark.gpu


def _engines(name, graphs=True, max_batch=8):
    cfg = get_model_config(name)
    sd = W.synth_hf_state_dict(cfg, seed=5, dtype=torch.float32)
    e_cpu = LLMEngine(EngineConfig(model=name, dtype="float32", device="cpu", max_batch=max_batch,
                                   max_seq_len=512, use_graphs=False),
                      ModelStage(cfg, 0, cfg.num_layers, "cpu", torch.float32).load_hf_state(sd))
    e_gpu = LLMEngine(EngineConfig(model=name, dtype="bfloat16", device="cuda", max_batch=max_batch,
                                   max_seq_len=512, use_graphs=graphs, num_kv_blocks=256,
                                   graph_batch_sizes=(1, 2, 4, 8)),
                      ModelStage(cfg, 0, cfg.num_layers, "cuda", torch.bfloat16).load_hf_state(sd))
    return e_cpu, e_gpu


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-llama-d128", "tiny-gpt2", "tiny-mixtral"])
def test_prefill_logits_gpu_vs_cpu(cuda, name):
    e_cpu, e_gpu = _engines(name, graphs=False)
    prompts = [[1, 5, 9, 200, 37, 44, 45, 46, 47, 48], [3, 4], list(range(10, 80))]
    outs = []
    for eng in (e_cpu, e_gpu):
        for p in prompts:
            eng.add_request(p, SamplingParams(max_new_tokens=1))
        st = eng.scheduler.schedule(0)
        hb = build_host_batch(st, eng.bm, 32)
        outs.append(eng.runner.execute(hb).float().cpu())
    torch.testing.assert_close(outs[1], outs[0], atol=5e-2, rtol=5e-2)


@pytest.mark.parametrize("name", ["tiny-llama", "tiny-mixtral"])
def test_graph_decode_matches_eager(cuda, name):
    _, e_eager = _engines(name, graphs=False)
    _, e_graph = _engines(name, graphs=True)
    prompts = [[1, 5, 9, 200], [3, 4, 7], list(range(10, 70)), [8] * 33, [9, 9, 9]]
    p = SamplingParams(max_new_tokens=24, ignore_eos=True)
    a = e_eager.generate(prompts, p)
    b = e_graph.generate(prompts, p)
    assert a == b
    assert e_graph.runner.graphs.graphs, "decode never went through a captured graph"


def test_native_kernels_used(cuda):
    assert _ext.kernels().arch == "gfx950"


@pytest.mark.parametrize("graphs", [True, False])
def test_lookahead_decode_matches_synchronous(cuda, graphs):
    """Lookahead (next decode issued before the in-flight step's tokens reach the host, input ids
    gathered on device) generates exactly what the synchronous loop does: sequences finishing by
    length at different steps (device gather path) and by EOS (a throw-away row in flight)."""
    prompts = [[1, 5, 9, 200], [3, 4, 7], list(range(10, 70)), [8] * 33, [9, 9, 9], [2, 3]]
    lens = [5, 17, 24, 9, 24, 2]

    def run(lookahead, eos=None):
        _, eng = _engines("tiny-llama", graphs=graphs)
        eng.lookahead = lookahead
        if eos is not None:
            eng.mcfg.eos_token_id = eos
        seqs = [eng.add_request(p, SamplingParams(max_new_tokens=n, ignore_eos=eos is None))
                for p, n in zip(prompts, lens)]
        eng.run_until_done()
        return [s.output for s in seqs], eng.num_lookahead

    sync, n0 = run(False)
    la, n1 = run(True)
    assert n0 == 0 and n1 > 0, "lookahead path never taken"
    assert la == sync
    # an EOS id that one sequence produces mid-way (and stops at) in the synchronous run
    eos = sync[2][7]
    sync_e, _ = run(False, eos)
    la_e, _ = run(True, eos)
    assert la_e == sync_e
    assert any(len(o) < n for o, n in zip(sync_e, lens)), "EOS never fired"


@pytest.mark.parametrize("attn", [4, 6, 7, 9])
@pytest.mark.parametrize("name", ["tiny-llama-d128", "tiny-mixtral"])
def test_chunked_prefill_gpu_matches_cpu_logits(cuda, name, attn):
    """A 300-token prompt prefilled in 64-token chunks on the GPU (each chunk's attention reads the
    earlier chunks from the paged cache) vs the CPU fp32 whole-prompt prefill: the last chunk's
    logits agree."""
    cfg = get_model_config(name)
    sd = W.synth_hf_state_dict(cfg, seed=5, dtype=torch.float32)
    prompt = [(13 * j) % 400 + 3 for j in range(300)]
    e_cpu = LLMEngine(EngineConfig(model=name, dtype="float32", device="cpu", max_batch=2, max_seq_len=512,
                                   use_graphs=False),
                      ModelStage(cfg, 0, cfg.num_layers, "cpu", torch.float32).load_hf_state(sd))
    e_gpu = LLMEngine(EngineConfig(model=name, dtype="bfloat16", device="cuda", max_batch=2, max_seq_len=512,
                                   use_graphs=False, num_kv_blocks=64, max_prefill_tokens=64),
                      ModelStage(cfg, 0, cfg.num_layers, "cuda", torch.bfloat16).load_hf_state(sd))
    logits = []
    from distributed_llms_amd import knobs
    for eng in (e_cpu, e_gpu):
        eng.add_request(prompt, SamplingParams(max_new_tokens=1))
        while True:
            st = eng.scheduler.schedule(0)
            with knobs.override(prefill_attn=attn):
                out = eng.runner.execute(build_host_batch(st, eng.bm, 32))
            final = st.seqs[0].chunk == 0
            eng.scheduler.complete(st, [0])
            if final:
                logits.append(out.float().cpu())
                break
    torch.testing.assert_close(logits[1], logits[0], atol=6e-2, rtol=5e-2)


def test_long_prompt_prefill_default_kernel_matches_cpu_logits(cuda):
    """The default prefill attention choice (knobs.prefill_attn = 0: the persistent 32x32x16 kernel
    from knobs.prefill_w32_min_q query rows at head_dim 128) on a 600-token prompt prefilled in one step, with the
    q-RoPE inside the kernel: logits vs the CPU fp32 prefill."""
    from distributed_llms_amd import knobs, ops
    name = "tiny-llama-d128"
    cfg = get_model_config(name)
    assert ops.prefill_attn_version(600, cfg.head_dim) == 9 and knobs.K.prefill_attn == 0
    sd = W.synth_hf_state_dict(cfg, seed=6, dtype=torch.float32)
    prompt = [(17 * j) % 450 + 5 for j in range(600)]
    e_cpu = LLMEngine(EngineConfig(model=name, dtype="float32", device="cpu", max_batch=2, max_seq_len=1024,
                                   use_graphs=False),
                      ModelStage(cfg, 0, cfg.num_layers, "cpu", torch.float32).load_hf_state(sd))
    e_gpu = LLMEngine(EngineConfig(model=name, dtype="bfloat16", device="cuda", max_batch=2, max_seq_len=1024,
                                   use_graphs=False, num_kv_blocks=64, max_prefill_tokens=1024),
                      ModelStage(cfg, 0, cfg.num_layers, "cuda", torch.bfloat16).load_hf_state(sd))
    logits = []
    for eng in (e_cpu, e_gpu):
        eng.add_request(prompt, SamplingParams(max_new_tokens=1))
        st = eng.scheduler.schedule(0)
        assert st.is_prefill and st.seqs[0].chunk == 0            # the whole prompt in one step
        logits.append(eng.runner.execute(build_host_batch(st, eng.bm, 32)).float().cpu())
    torch.testing.assert_close(logits[1], logits[0], atol=6e-2, rtol=5e-2)


def test_mixed_prefill_decode_steps_gpu(cuda):
    """Arrivals during decode ride along with the running rows (mixed steps, eager prefill path with
    split decode / prefill attention) on the HIP kernels.  Batch composition changes the GEMMs'
    split-K counts, so bf16 greedy outputs may part at near-ties: most sequences must match the
    prefill-first schedule exactly, every sequence must finish with the right length."""
    import numpy as np
    from distributed_llms_amd.config import EngineConfig
    from distributed_llms_amd.engine.llm_engine import LLMEngine
    from distributed_llms_amd.engine.sequence import SamplingParams

    def run(mixed):
        eng = LLMEngine(EngineConfig(model="synthetic:tiny-llama-d128", max_batch=16, max_seq_len=256,
                                     num_kv_blocks=256, mixed_prefill_tokens=mixed, graph_batch_sizes=(4, 8, 16)))
        rng = np.random.default_rng(5)
        prompts = [rng.integers(3, 500, size=int(rng.integers(8, 60))).tolist() for _ in range(14)]
        p = SamplingParams(max_new_tokens=12, ignore_eos=True)
        seqs, i, step = [], 0, 0
        waves = [(0, 4), (3, 4), (6, 3), (10, 3)]
        while waves or eng.has_work():
            while waves and waves[0][0] <= step:
                _, n = waves.pop(0)
                seqs += [eng.add_request(q, p) for q in prompts[i:i + n]]
                i += n
            eng.step()
            step += 1
        return [s.output for s in seqs], eng.scheduler.num_mixed

    ref, n0 = run(0)
    out, n1 = run(64)
    assert n0 == 0 and n1 > 0
    assert all(len(o) == 12 for o in out)
    assert sum(a == b for a, b in zip(out, ref)) >= 11, (out, ref)


def test_prefill_with_block_table_wider_than_lds_kernel(cuda):
    """A prefill whose block table is wider than the LDS prefill kernel stages (> 1024 blocks, i.e.
    sequences past 32k tokens) must not take the in-kernel q-RoPE path: the launcher falls back to
    the register-tiled kernel, which reads a rotated q.  The stage then appends with write_q=True
    and runs the plain prefill kernel -- same logits as the narrow table, within the kernels' bf16
    difference."""
    from distributed_llms_amd import knobs, ops
    assert not ops.prefill_rope_in_attention(ops.PF_MAX_CHUNKS + 1)
    _, e_gpu = _engines("tiny-llama-d128", graphs=False)
    prompts = [[1, 5, 9, 200, 37, 44, 45, 46, 47, 48], list(range(10, 80))]
    for p in prompts:
        e_gpu.add_request(p, SamplingParams(max_new_tokens=1))
    st = e_gpu.scheduler.schedule(0)
    outs = []
    with knobs.override(prefill_attn=4, prefill_fused_rope=True):
        for width in (None, ops.PF_MAX_CHUNKS + 76):
            hb = build_host_batch(st, e_gpu.bm, 32, max_blocks=width)
            if width is not None:
                assert hb.block_tables.shape[1] == width
            outs.append(e_gpu.runner.execute(hb).float().cpu())
    torch.testing.assert_close(outs[1], outs[0], atol=3e-2, rtol=3e-2)
