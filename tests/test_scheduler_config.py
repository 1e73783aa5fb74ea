"""CPU unit tests: EngineConfig parsing/validation, the native paged-KV
block manager, the continuous-batching scheduler driven with a fake clock, and request metrics.

The reference has none of these (no config system, no KV cache, a FIFO queue with 0.1 s polling:
SURVEY §2.7, §2.9 D15-D17); its test suite is four unittest files."""
import json

import numpy as np
import pytest

from distributed_llms_amd.config import EngineConfig, get_model_config
from distributed_llms_amd.engine.batch import HostBatch, build_decode_batch, build_host_batch
from distributed_llms_amd.engine.llm_engine import make_block_manager
from distributed_llms_amd.engine.scheduler import Scheduler
from distributed_llms_amd.engine.sequence import SamplingParams, Sequence, SeqStatus
from distributed_llms_amd.utils.metrics import RequestMetrics, itl_stats, percentile, prometheus_text


# ------------------------------------------------------------------ config
def test_config_json_yaml_roundtrip_and_overrides(tmp_path):
    c = EngineConfig(model="synthetic:tiny-llama", num_workers=2, max_batch=32, graph_batch_sizes=(1, 8, 32))
    p = tmp_path / "c.json"
    p.write_text(json.dumps(c.to_dict()))
    c2 = EngineConfig.from_file(str(p))
    assert c2 == c and isinstance(c2.graph_batch_sizes, tuple)
    y = tmp_path / "c.yaml"
    y.write_text("model: synthetic:tiny-llama\nmax_batch: 7\nkv_block_size: 16\n")
    c3 = EngineConfig.from_file(str(y))
    assert (c3.max_batch, c3.kv_block_size) == (7, 16)
    c4 = c3.apply_overrides(max_batch=9, port=None)       # None = "not given on the CLI"
    assert c4.max_batch == 9 and c4.port == c3.port


@pytest.mark.parametrize("bad", [{"dtype": "int8"}, {"kv_block_size": 24}, {"num_workers": 0},
                                 {"max_batch": 0}, {"num_workers": 99}, {"transport": "tcp"},
                                 {"comm_timeout_s": 0}])
def test_config_validation_rejects(bad):
    with pytest.raises(ValueError):
        EngineConfig(model="synthetic:tiny-llama", **bad).validate()


def test_config_unknown_key_and_presets():
    with pytest.raises(ValueError):
        EngineConfig.from_dict({"modle": "x"})
    for name, layers, hkv in [("llama3-8b", 32, 8), ("llama3-70b", 80, 8), ("mixtral-8x7b", 32, 8),
                              ("gpt2-small", 12, 12)]:
        m = get_model_config(f"synthetic:{name}")
        assert (m.num_layers, m.num_kv_heads) == (layers, hkv)
    a, b = get_model_config("llama3-8b"), get_model_config("llama3-8b")
    a.eos_token_id = -5
    assert b.eos_token_id != -5                              # presets are copied, never shared


# ------------------------------------------------------------------ block manager
def test_block_manager_alloc_lifo_and_metadata():
    bm = make_block_manager(10, 4)                  # block 0 = scratch
    assert bm.num_free() == 9
    assert bm.ensure_capacity(1, 9)                 # 3 blocks
    assert bm.ensure_capacity(2, 4)                 # 1 block
    assert not bm.ensure_capacity(3, 100)           # all-or-nothing
    assert bm.num_free() == 5
    t1 = bm.block_table(1)
    bm.free_sequence(1)
    assert bm.ensure_capacity(4, 1)
    assert bm.block_table(4) == [t1[0]]             # LIFO: most recently freed first
    slots = np.empty(3, np.int32)
    n = bm.fill_slots(np.array([2, 4], np.int64), np.array([2, 0], np.int32), np.array([2, 1], np.int32), slots)
    b2 = bm.block_table(2)[0]
    assert n == 3 and slots.tolist() == [b2 * 4 + 2, b2 * 4 + 3, t1[0] * 4]
    bt = np.full((2, 3), -7, np.int32)
    bm.fill_block_tables(np.array([2, 4], np.int64), bt, 0)
    assert bt[:, 1:].tolist() == [[0, 0], [0, 0]]
    with pytest.raises(Exception):
        bm.fill_slots(np.array([2], np.int64), np.array([4], np.int32), np.array([1], np.int32), slots)
    assert bm.ensure_capacity_batch(np.array([2, 4], np.int64), np.array([8, 8], np.int64)) == -1


# ------------------------------------------------------------------ scheduler
def _seq(n, max_new=3, eos=None, ignore_eos=True):
    return Sequence(list(range(1, n + 1)), SamplingParams(max_new_tokens=max_new, ignore_eos=ignore_eos),
                    eos_token_id=eos)


def test_scheduler_prefill_then_decode_fake_clock():
    bm = make_block_manager(64, 4)
    sch = Scheduler(bm, num_slots=1, max_batch=4, max_prefill_tokens=10, max_seq_len=64)
    seqs = [_seq(4), _seq(4), _seq(4)]
    for s in seqs:
        s.arrival = 100.0
        sch.add(s)
    st = sch.schedule(0)                                       # prefill bounded by 10 tokens -> 2 seqs
    assert st.is_prefill and [s.seq_id for s in st.seqs] == [seqs[0].seq_id, seqs[1].seq_id]
    assert sch.complete(st, [7, 8], now=100.5) == []
    assert seqs[0].ttft() == pytest.approx(0.5)
    st = sch.schedule(0)                                       # waiting seq admitted before decode
    assert st.is_prefill and st.seqs == [seqs[2]]
    sch.complete(st, [9], now=101.0)
    st = sch.schedule(0)
    assert not st.is_prefill and len(st.seqs) == 3 and st.num_tokens == 3
    hb = build_host_batch(st, bm, 4, 16)
    assert hb.ids.tolist() == [7, 8, 9] and hb.positions.tolist() == [4, 4, 4]
    assert HostBatch.unpack(hb.pack()).slots.tolist() == hb.slots.tolist()
    # the lookahead builder produces the same metadata from arrays
    ids = np.array([s.seq_id for s in st.seqs], np.int64)
    hb2 = build_decode_batch(ids, np.array([s.total_len for s in st.seqs], np.int32), bm, 4, 16)
    assert hb2.slots.tolist() == hb.slots.tolist() and (hb2.block_tables == hb.block_tables).all()
    sch.complete(st, [1, 2, 3], now=102.0)
    st = sch.schedule(0)
    done = sch.complete(st, [4, 5, 6], now=103.0)              # third token -> max_new_tokens reached
    assert {s.seq_id for s in done} == {s.seq_id for s in seqs}
    assert seqs[0].output == [7, 1, 4] and seqs[0].finish_reason == "length"
    assert seqs[0].latency() == pytest.approx(3.0) and seqs[0].itl() == pytest.approx([1.5, 1.0])
    assert bm.num_free() == 63 and not sch.has_work()


def test_scheduler_eos_abort_and_slot_balance():
    bm = make_block_manager(64, 4)
    sch = Scheduler(bm, num_slots=2, max_batch=4, max_prefill_tokens=100, max_seq_len=64)
    a, b, c = _seq(3, 10, eos=42, ignore_eos=False), _seq(3, 10), _seq(3, 10)
    for s in (a, b, c):
        sch.add(s)
    st0 = sch.schedule(0)
    assert st0.seqs == [a, b]                                   # slot 0 takes its even share (2 of 3)
    sch.complete(st0, [42, 5])                                  # a: EOS on its first token
    assert a.finished and a.finish_reason == "eos"
    d = _seq(3, 10)
    sch.add(d)
    st0 = sch.schedule(0)                                       # share = ceil((1 running + 2 waiting) / 2)
    assert st0.is_prefill and st0.seqs == [c]                   # slot 0 tops up to 2
    st1 = sch.schedule(1)
    assert st1.is_prefill and st1.seqs == [d]                   # the emptier slot takes the rest
    sch.complete(st0, [3])
    assert sch.schedule(0).is_prefill is False and sch.running[0] == [b, c]
    assert sch.abort(b.seq_id) and b.status is SeqStatus.ABORTED
    assert not sch.abort(12345)


def test_burst_is_spread_over_slots_in_full_prefill_chunks():
    """A burst of 8 requests over 2 slots with a 2-request prefill budget: each slot tops itself
    up to its share of 4 in prefill chunks before decoding (no early decode at a quarter batch)."""
    bm = make_block_manager(256, 4)
    sch = Scheduler(bm, num_slots=2, max_batch=8, max_prefill_tokens=8, max_seq_len=64)
    seqs = [_seq(4, 10) for _ in range(8)]
    for s in seqs:
        sch.add(s)
    kinds = []
    for rnd in range(3):
        for slot in (0, 1):
            st = sch.schedule(slot)
            kinds.append((slot, st.is_prefill, st.size))
            sch.complete(st, [1] * st.size)
    assert kinds == [(0, True, 2), (1, True, 2), (0, True, 2), (1, True, 2), (0, False, 4), (1, False, 4)]
    assert sch.num_prefilling == 0 and not sch.waiting


def test_scheduler_preempts_youngest_when_kv_runs_out():
    bm = make_block_manager(5, 4)                               # 4 usable blocks
    sch = Scheduler(bm, num_slots=1, max_batch=4, max_prefill_tokens=100, max_seq_len=64)
    old, young = _seq(7, 20), _seq(7, 20)
    sch.add(old)
    sch.add(young)
    st = sch.schedule(0)
    sch.complete(st, [1, 1])                                    # 8 tokens each: 2 blocks each, pool full
    st = sch.schedule(0)                                        # decode at position 7: still 2 blocks
    assert len(st.seqs) == 2
    sch.complete(st, [2, 2])
    st = sch.schedule(0)                                        # position 8 needs a 3rd block -> preempt young
    assert [s.seq_id for s in st.seqs] == [old.seq_id]
    assert sch.num_preemptions == 1 and young.status is SeqStatus.WAITING and young.num_cached == 0
    assert sch.waiting[0] is young


def test_too_long_prompt_is_rejected_not_scheduled():
    sch = Scheduler(make_block_manager(8, 4), max_seq_len=8)
    s = _seq(8)
    sch.add(s)
    assert s.finish_reason == "too_long" and sch.pop_finished() == [s] and sch.schedule(0) is None


# ------------------------------------------------------------------ metrics
def test_metrics_percentiles_and_prometheus():
    assert percentile([], 50) is None
    assert percentile([1, 2, 3, 4], 50) == pytest.approx(2.5)
    m = RequestMetrics()
    for i in range(10):
        m.record(5, 0.1 * (i + 1), 0.01)
    s = m.summary()
    assert s["requests"] == 10 and s["output_tokens"] == 50
    assert s["latency_p50_s"] == pytest.approx(0.55) and s["latency_p99_s"] == pytest.approx(0.991)
    txt = prometheus_text(s)
    assert "# TYPE dllm_latency_p50_s gauge" in txt and "dllm_requests 10" in txt
    seq = _seq(2)
    seq.token_times = [1.0, 1.25, 1.75]
    assert itl_stats([seq])["itl_p50_s"] == pytest.approx(0.375)


# ------------------------------------------------------------------ master placement
def _master_with(workers_mem, model="synthetic:llama3-70b", shards=2):
    from distributed_llms_amd.master.node import MasterNode
    m = MasterNode(config=EngineConfig(model=model))
    m.initialize_model(model, shards)
    for i, mem in enumerate(workers_mem):
        m.workers[f"w{i}"] = {"capabilities": {"memory": mem}}
    return m


def test_assign_shards_capacity_aware():
    gib = 2 ** 30
    # homogeneous node: registration order
    m = _master_with([288 * gib] * 3, shards=2)
    assert m.assign_shards() == {"w0": [0], "w1": [1]}
    assert sum(m.stage_weight_bytes()) > 125 * gib            # 70B bf16 is ~139-141 GB over the stages
    # heterogeneous: the small device is skipped when a larger one is free
    m = _master_with([288 * gib, 24 * gib, 288 * gib], shards=2)
    assert set(m.assign_shards()) == {"w0", "w2"}
    # nothing can hold a 70 GB stage
    m = _master_with([48 * gib, 48 * gib], shards=2)
    with pytest.raises(ValueError, match="needs"):
        m.assign_shards()
    # CPU workers (memory 0): plain registration order, no capacity check
    m = _master_with([0, 0], model="synthetic:gpt2-small", shards=2)
    assert m.assign_shards() == {"w0": [0], "w1": [1]}


def test_chunked_prefill_of_a_long_prompt():
    """A prompt longer than max_prefill_tokens is prefilled in chunks over several steps (each
    attending to the KV its earlier chunks cached); only the last chunk's token counts."""
    bm = make_block_manager(64, 4)
    sch = Scheduler(bm, num_slots=1, max_batch=4, max_prefill_tokens=40, max_seq_len=256)
    sch.MIN_CHUNK = 8
    long_, short = _seq(100, 3), _seq(10, 3)
    sch.add(long_)
    sch.add(short)
    st = sch.schedule(0)
    assert st.is_prefill and st.seqs == [long_] and long_.chunk == 40 and st.num_tokens == 40
    hb = build_host_batch(st, bm, 4)
    assert hb.positions.tolist() == list(range(40)) and hb.seq_lens.tolist() == [40]
    assert sch.complete(st, [99]) == [] and long_.output == [] and long_.num_cached == 40
    assert sch.waiting[0] is long_
    st = sch.schedule(0)
    hb = build_host_batch(st, bm, 4)
    assert st.seqs == [long_] and hb.positions[0] == 40 and hb.seq_lens.tolist() == [80]
    sch.complete(st, [98])
    st = sch.schedule(0)                                # the last 20 tokens + the short prompt
    assert st.seqs == [long_, short] and long_.chunk == 0 and st.num_tokens == 30
    hb = build_host_batch(st, bm, 4)
    assert hb.seq_lens.tolist() == [100, 10] and hb.logits_idx.tolist() == [19, 29]
    sch.complete(st, [5, 6])
    assert long_.output == [5] and short.output == [6] and sch.num_running() == 2
    assert bm.block_table(long_.seq_id) and len(bm.block_table(long_.seq_id)) == 25


def test_abort_of_a_partly_prefilled_prompt_frees_its_blocks():
    bm = make_block_manager(64, 4)
    sch = Scheduler(bm, num_slots=1, max_batch=4, max_prefill_tokens=16, max_seq_len=256)
    s = _seq(50, 3)
    sch.add(s)
    sch.complete(sch.schedule(0), [1])
    assert s.num_cached == 16 and bm.num_free() == 63 - 4
    assert sch.abort(s.seq_id) and bm.num_free() == 63


def test_partial_prompts_on_two_slots_do_not_deadlock_a_tight_pool():
    """two long prompts chunk-prefilled on two slots can each hold part of a pool too
    small for both; with nothing running, the scheduler must drop the other prompt's cached chunks
    (recomputed later) instead of returning None forever."""
    bm = make_block_manager(11, 4)                              # 10 usable blocks = 40 tokens
    sch = Scheduler(bm, num_slots=2, max_batch=4, max_prefill_tokens=16, max_seq_len=64)
    sch.MIN_CHUNK = 4
    a, b = _seq(30, 2), _seq(30, 2)
    sch.add(a)
    sch.add(b)
    sa, sb = sch.schedule(0), sch.schedule(1)
    assert sa.seqs == [a] and sb.seqs == [b] and a.chunk == 16 and b.chunk == 16
    sch.complete(sa, [0])
    sch.complete(sb, [0])
    assert bm.num_free() == 2 and a.num_cached == 16 and b.num_cached == 16
    steps = 0
    while sch.has_work():
        progressed = False
        for slot in (0, 1):
            st = sch.schedule(slot)
            if st is not None:
                sch.complete(st, [7] * st.size)
                progressed = True
        assert progressed, "scheduler stalled with work left"
        steps += 1
        assert steps < 100
    fin = sch.pop_finished()
    assert sorted(s.seq_id for s in fin) == sorted([a.seq_id, b.seq_id])
    assert all(s.finish_reason == "length" and len(s.output) == 2 for s in fin)
    assert bm.num_free() == 10


def test_prompt_larger_than_the_whole_pool_is_finished_not_spun():
    bm = make_block_manager(5, 4)                               # 16 tokens of KV
    sch = Scheduler(bm, num_slots=1, max_batch=4, max_prefill_tokens=8, max_seq_len=64)
    sch.MIN_CHUNK = 4
    s = _seq(30, 2)
    sch.add(s)
    for _ in range(4):
        st = sch.schedule(0)
        if st is None:
            break
        sch.complete(st, [0])
    assert s.finish_reason == "kv_capacity" and not sch.has_work() and bm.num_free() == 4


def test_master_plans_carry_the_unit_group(monkeypatch):
    """a sub-layer (group 5) plan set on the master must reach the workers with its
    group, or they would read atom ranges as half-layer units."""
    m = _master_with([0, 0], model="synthetic:gpt2-small", shards=2)
    m.assign_shards()
    plans = m._plans()
    assert all(p["unit_group"] == 2 for p in plans)
    monkeypatch.setenv("DLLM_PP_UNITS", "5:0,31;31,60")
    plans = m._plans()
    assert [p["unit_group"] for p in plans] == [5, 5]
    assert [p["unit_range"] for p in plans] == [[0, 31], [31, 60]]
    assert [p["layer_range"] for p in plans] == [[0, 7], [6, 12]]


def test_reduced_depth_preset_keeps_layer_shapes():
    """``<preset>@<N>l``: a preset's full-size layer dimensions at N layers (GPU tests and one-GPU
    pipeline rehearsals of the 70B / Mixtral configs)."""
    from distributed_llms_amd.config import PRESETS, get_model_config
    c = get_model_config("synthetic:llama3-70b@4l")
    full = PRESETS["llama3-70b"]
    assert c.num_layers == 4 and c.name == "llama3-70b@4l"
    assert (c.hidden_size, c.intermediate_size, c.num_heads, c.num_kv_heads, c.vocab_size) == \
        (full.hidden_size, full.intermediate_size, full.num_heads, full.num_kv_heads, full.vocab_size)
    assert get_model_config("mixtral-8x7b@2l").num_experts == 8
    with pytest.raises(KeyError):
        get_model_config("llama3-70b@x")
