"""Mixed prefill + decode steps (prefill chunks interleave with decode microbatches).

Requests that arrive while a slot decodes are prefilled in chunks of at most
``EngineConfig.mixed_prefill_tokens`` tokens riding along with the slot's decode rows, instead of a
prefill-only step that stalls every running sequence.  CPU (fp32 reference ops): the mixed
schedule must generate exactly what the prefill-first schedule generates, and the scheduler must
keep every step's prompt tokens within the budget."""
import numpy as np
import pytest
import torch

from distributed_llms_amd.config import EngineConfig
from distributed_llms_amd.engine.batch import HostBatch, build_host_batch
from distributed_llms_amd.engine.llm_engine import LLMEngine, make_block_manager
from distributed_llms_amd.engine.scheduler import Scheduler
from distributed_llms_amd.engine.sequence import SamplingParams, Sequence


def _prompts(n, seed=0, lo=5, hi=40):
    rng = np.random.default_rng(seed)
    return [rng.integers(3, 200, size=int(rng.integers(lo, hi))).tolist() for _ in range(n)]


def _staggered(mixed, arrivals=((0, 3), (2, 4), (5, 3), (9, 5)), gen=10, model="tiny-llama"):
    """Feed requests in waves (after `step` engine steps, `n` new prompts); return outputs, engine."""
    eng = LLMEngine(EngineConfig(model=f"synthetic:{model}", device="cpu", dtype="float32", max_batch=16,
                                 max_seq_len=128, use_graphs=False, num_kv_blocks=256, mixed_prefill_tokens=mixed))
    p = SamplingParams(max_new_tokens=gen, ignore_eos=True)
    prompts = _prompts(sum(n for _, n in arrivals))
    seqs, i, step, waves = [], 0, 0, list(arrivals)
    while waves or eng.has_work():
        while waves and waves[0][0] <= step:
            _, n = waves.pop(0)
            seqs += [eng.add_request(q, p) for q in prompts[i:i + n]]
            i += n
        eng.step()
        step += 1
    return [s.output for s in seqs], eng


@pytest.mark.parametrize("budget", [8, 64])
def test_mixed_steps_reproduce_prefill_first(budget):
    ref, e0 = _staggered(0)
    out, e1 = _staggered(budget)
    assert e0.scheduler.num_mixed == 0
    assert e1.scheduler.num_mixed > 0             # arrivals during decode did ride along
    assert out == ref


def test_mixed_step_budget_and_order():
    bm = make_block_manager(64, 4)
    sch = Scheduler(bm, num_slots=1, max_batch=8, max_prefill_tokens=100, max_seq_len=64, mixed_prefill_tokens=6)
    a = Sequence([1, 2, 3], SamplingParams(max_new_tokens=5, ignore_eos=True))
    sch.add(a)
    st = sch.schedule(0)
    assert st.is_prefill and not st.mixed
    sch.complete(st, [7])
    b = Sequence(list(range(10, 24)), SamplingParams(max_new_tokens=3, ignore_eos=True))   # 14 tokens
    sch.add(b)
    st = sch.schedule(0)
    assert st.mixed and list(st.rows) == [a.seq_id] and st.seqs == [b]
    assert st.num_tokens == 1 + 6 and st.size == 2    # one decode row + a 6-token chunk of b
    hb = build_host_batch(st, bm, 4, None, 3)
    assert hb.num_decode == 1 and hb.is_prefill
    assert list(hb.cu_seqlens) == [0, 1, 7] and list(hb.logits_idx) == [0, 6]
    assert hb.positions[0] == 3 and list(hb.positions[1:]) == list(range(0, 6))
    rt = HostBatch.unpack(hb.pack())
    assert rt.num_decode == 1 and np.array_equal(rt.block_tables, hb.block_tables)
    sch.complete(st, np.array([8, 99], np.int32))     # b's token is discarded (non-final chunk)
    assert b.num_cached == 6 and b in sch.waiting and b.output == []
    st = sch.schedule(0)
    assert st.mixed and st.num_tokens == 1 + 6
    sch.complete(st, np.array([9, 99], np.int32))
    st = sch.schedule(0)                              # last 2 tokens of b: the final chunk
    assert st.mixed and st.num_tokens == 1 + 2
    sch.complete(st, np.array([10, 42], np.int32))
    assert b.output == [42]
    st = sch.schedule(0)                              # nothing waiting: a plain decode step
    assert not st.is_prefill and st.size == 2


def test_mixed_steps_under_tensor_metadata_roundtrip():
    """A mixed HostBatch survives the wire format the pipeline / TP followers receive."""
    bm = make_block_manager(32, 4)
    sch = Scheduler(bm, 1, 8, 100, 64, mixed_prefill_tokens=16)
    for q in ([1, 2], [3, 4, 5]):
        sch.add(Sequence(q, SamplingParams(max_new_tokens=4, ignore_eos=True, temperature=0.5, top_k=3)))
    st = sch.schedule(0)
    sch.complete(st, [5, 6])
    sch.add(Sequence([9, 9, 9, 9], SamplingParams(max_new_tokens=2)))
    st = sch.schedule(0)
    assert st.mixed
    hb = build_host_batch(st, bm, 4, None, 0)
    rt = HostBatch.unpack(hb.pack())
    for f in ("ids", "positions", "slots", "seq_lens", "cu_seqlens", "logits_idx", "sampling"):
        assert np.array_equal(getattr(rt, f), getattr(hb, f)), f
    assert rt.sampling.shape == (3, 3) and rt.sampling[2, 0] == 0        # the greedy newcomer


def test_mixed_steps_pipeline_loopback():
    """The pipeline driver runs the same mixed steps through its stages (followers unpack the
    decode-row count from the wire header)."""
    from distributed_llms_amd.parallel.pipeline import run_loopback_pipeline
    ecfg = EngineConfig(model="synthetic:tiny-llama", device="cpu", dtype="float32", max_batch=8, max_seq_len=128,
                        use_graphs=False, num_kv_blocks=256, mixed_prefill_tokens=16)
    prompts = _prompts(6, seed=3)
    p = SamplingParams(max_new_tokens=8, ignore_eos=True)
    ref = LLMEngine(ecfg).generate(prompts, p)
    outs, drv, _ = run_loopback_pipeline(ecfg, 2, prompts, p, device="cpu")
    assert outs == ref


def test_mixed_budget_capped_by_prefill_budget():
    bm = make_block_manager(64, 4)
    sch = Scheduler(bm, 1, 8, max_prefill_tokens=100, max_seq_len=64, mixed_prefill_tokens=8192)
    assert sch.mixed_prefill_tokens == 100
    assert Scheduler(bm, 1, 8, 100, 64, mixed_prefill_tokens=0).mixed_prefill_tokens == 0


def test_mixed_step_total_tokens_within_prefill_budget():
    """Decode rows + prompt tokens of a mixed step never exceed max_prefill_tokens (the pipeline's
    hop slots and prefill buffers are sized for it)."""
    bm = make_block_manager(256, 4)
    sch = Scheduler(bm, 1, 16, max_prefill_tokens=40, max_seq_len=64, mixed_prefill_tokens=8192)
    for _ in range(3):
        sch.add(Sequence([1] * 10, SamplingParams(max_new_tokens=20, ignore_eos=True)))
    st = sch.schedule(0)
    assert st.is_prefill and not st.mixed and st.num_tokens == 30
    sch.complete(st, [5, 5, 5])
    for _ in range(6):
        sch.add(Sequence([2] * 12, SamplingParams(max_new_tokens=4, ignore_eos=True)))
    while sch.waiting:
        st = sch.schedule(0)
        if st.mixed:
            assert st.num_tokens <= 40, st.num_tokens
        sch.complete(st, [7] * st.size)
    assert sch.num_mixed > 0
