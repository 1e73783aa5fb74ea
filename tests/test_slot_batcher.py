"""Native decode-step bookkeeping (csrc/runtime/slot_batcher.cpp) vs the Python reference
builder (engine/batch.py::build_decode_batch) and the scheduler's stop rules.  CPU only."""
import numpy as np
import pytest

from distributed_llms_amd import _ext
from distributed_llms_amd.engine.batch import HostBatch, build_decode_batch
from distributed_llms_amd.engine.llm_engine import make_block_manager


def _setup(nseq=5, plen=9, bs=4, max_seq=64, remaining=10, eos=-1, nb=128):
    bm = make_block_manager(nb, bs)
    sb = _ext.runtime().SlotBatcher(bm, 2, max_seq)
    ids = list(range(100, 100 + nseq))
    for i, s in enumerate(ids):
        assert bm.ensure_capacity(s, plen + i)
        sb.admit(0, s, plen + i, 50 + i, remaining, eos)
    return bm, sb, ids


def test_sync_decode_matches_python_builder():
    bm, sb, ids = _setup()
    packed, rows, keep = sb.build_decode(0, 16, 7, False)
    assert rows.tolist() == ids and keep is None
    hb = HostBatch.unpack(packed)
    ref = build_decode_batch(np.array(ids, np.int64), np.array([9 + i for i in range(5)], np.int32), bm, 4, 16,
                             step_id=7)
    assert not hb.is_prefill and hb.step_id == 7 and hb.max_q_len == 1 and hb.max_ctx == 13
    assert hb.ids.tolist() == [50 + i for i in range(5)]
    for f in ("positions", "slots", "seq_lens", "cu_seqlens", "block_tables", "logits_idx"):
        assert np.array_equal(getattr(hb, f), getattr(ref, f)), f
    assert hb.sampling is None
    # the packed form round-trips through the Python codec
    assert np.array_equal(HostBatch.unpack(hb.pack()).slots, hb.slots)


def test_complete_appends_and_stops_by_length_and_eos():
    bm, sb, ids = _setup(nseq=3, remaining=2, eos=42)
    _, rows, _ = sb.build_decode(0, 16)
    assert sb.complete(0, rows, np.array([42, 5, 6], np.int32), 1.0) == 1      # EOS on row 0
    assert sb.take_finished() == [(100, "eos")]
    toks, times = sb.take_output(100)
    assert toks.tolist() == [42] and times.tolist() == [1.0]
    assert sb.num_running(0) == 2 and not bm.has_sequence(100)
    _, rows, _ = sb.build_decode(0, 16)
    assert rows.tolist() == [101, 102]
    assert sb.state(101)[:3] == (11, 1, 1)               # len, pending, remaining
    assert sb.complete(0, rows, np.array([7, 8], np.int32), 2.0) == 2          # remaining hit 0
    assert sorted(sb.take_finished()) == [(101, "length"), (102, "length")]
    assert sb.take_output(101)[0].tolist() == [5, 7] and sb.num_running_total() == 0


def test_max_seq_len_stop():
    bm = make_block_manager(64, 4)
    sb = _ext.runtime().SlotBatcher(bm, 1, 12)
    bm.ensure_capacity(1, 10)
    sb.admit(0, 1, 10, 3, 100)
    for k in range(2):
        _, rows, _ = sb.build_decode(0, 3)
        sb.complete(0, rows, np.array([k], np.int32), 0.0)
    assert sb.take_finished() == [(1, "max_seq_len")]


def test_lookahead_positions_keep_and_throwaway_rows():
    bm, sb, ids = _setup(nseq=3, remaining=2, eos=42)
    p1, r1, _ = sb.build_decode(0, 16)                     # step A in flight
    p2, r2, keep = sb.build_decode(0, 16, 1, True)         # step B built before A completes
    h1, h2 = HostBatch.unpack(p1), HostBatch.unpack(p2)
    assert r2.tolist() == ids and keep is None             # every row can still generate
    assert (h2.positions == h1.positions + 1).all() and (h2.seq_lens == h1.seq_lens + 1).all()
    assert h2.ids.tolist() == [0, 0, 0]                    # placeholders: ids come from the device
    # a third step is impossible: remaining = 2 is used up by the two in flight
    assert sb.build_decode(0, 16, 2, True) is None
    # A: row 0 hits EOS -> its B row is a throw-away
    assert sb.complete(0, r1, np.array([42, 1, 2], np.int32), 1.0) == 1
    sb.take_finished()
    sb.take_output(100)
    assert sb.complete(0, r2, np.array([9, 3, 4], np.int32), 2.0) == 2      # rows 1, 2 end by length
    assert {s for s, _ in sb.take_finished()} == {101, 102}
    assert sb.take_output(101)[0].tolist() == [1, 3]


def test_lookahead_leaves_out_length_finishers_and_reports_keep():
    bm = make_block_manager(64, 4)
    sb = _ext.runtime().SlotBatcher(bm, 1, 64)
    for s, rem in ((1, 1), (2, 5), (3, 5)):
        bm.ensure_capacity(s, 6)
        sb.admit(0, s, 6, 9, rem)
    _, r1, _ = sb.build_decode(0, 16)
    _, r2, keep = sb.build_decode(0, 16, 1, True)
    assert r1.tolist() == [1, 2, 3] and r2.tolist() == [2, 3] and keep.tolist() == [1, 2]


def test_lookahead_refuses_rows_the_previous_step_did_not_carry():
    bm, sb, ids = _setup(nseq=2)
    sb.build_decode(0, 16)
    bm.ensure_capacity(777, 5)
    sb.admit(0, 777, 5, 1, 3)                              # admitted after the step was built
    assert sb.build_decode(0, 16, 1, True) is None


def test_sync_decode_preempts_youngest():
    bm = make_block_manager(5, 4)                          # block 0 scratch: 4 usable
    sb = _ext.runtime().SlotBatcher(bm, 1, 64)
    for s in (1, 2):
        bm.ensure_capacity(s, 8)
        sb.admit(0, s, 8, 1, 20)
    _, rows, _ = sb.build_decode(0, 16)
    sb.complete(0, rows, np.array([5, 5], np.int32), 0.0)  # len 9: needs a third block each
    _, rows, _ = sb.build_decode(0, 16)
    assert rows.tolist() == [1] and sb.take_preempted() == [2]
    assert sb.take_output(2)[0].tolist() == [5] and not bm.has_sequence(2)


def test_sampling_block_and_abort():
    bm, sb, _ = _setup(nseq=1)
    bm.ensure_capacity(7, 4)
    sb.admit(0, 7, 4, 1, 5, -1, 7000, 40, 9000)
    hb = HostBatch.unpack(sb.build_decode(0, 16)[0])
    assert hb.sampling.tolist() == [[0, 0, 10000], [7000, 40, 9000]]
    assert hb.sampling_args()["temperatures"] == pytest.approx([0.0, 0.7])
    assert sb.abort(7) and not sb.abort(7) and sb.take_finished() == [(7, "abort")]
    assert not bm.has_sequence(7)


def test_misuse_raises():
    bm, sb, ids = _setup(nseq=1)
    with pytest.raises(Exception):
        sb.admit(0, ids[0], 5, 1, 3)                      # already registered
    with pytest.raises(Exception):
        sb.admit(5, 9, 5, 1, 3)                           # bad slot
    with pytest.raises(Exception):
        sb.take_output(ids[0])                            # still running
    sb.build_decode(0, 16)
    with pytest.raises(Exception):
        sb.build_decode(0, 16)                            # sync step with one in flight
