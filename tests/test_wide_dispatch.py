"""Decode GEMM routing between the wide-M HIP kernel (csrc/kernels/gemm_wide.hip) and hipBLASLt.

The cutovers are measured in-engine (profiles/wide_gemm.md): gate|up (SwiGLU) and qkv / o on the
wide kernel up to M = 256, the K >= 8192 down projection up to M = 512 (distributed_llms_amd/knobs.py).
CPU-only: `_use_wide` is pure shape / dtype logic."""
import pytest
import torch

from distributed_llms_amd.ops import gemm


def _xw(m, n, k):
    return torch.empty(m, k, dtype=torch.bfloat16), torch.empty(n, k, dtype=torch.bfloat16)


@pytest.fixture(autouse=True)
def _defaults():
    # pin the shipped defaults (a DLLM_KNOBS override in the environment cannot move the boundaries)
    from distributed_llms_amd import knobs
    saved = knobs.as_dict()
    for f, v in knobs.Knobs().__dict__.items():
        setattr(knobs.K, f, v)
    yield
    knobs.update(saved)


@pytest.mark.parametrize("m,expect", [(1, True), (64, True), (256, True), (257, False), (384, False), (512, False)])
def test_gate_up_cutover(m, expect):
    x, w = _xw(m, 2 * 14336, 4096)
    assert gemm._use_wide(m, w.shape[0], 4096, x, w, swiglu=True) is expect


@pytest.mark.parametrize("m,expect", [(1, True), (256, True), (384, True), (385, False), (512, False), (768, False)])
def test_down_cutover(m, expect):
    x, w = _xw(m, 4096, 14336)
    assert gemm._use_wide(m, 4096, 14336, x, w) is expect


@pytest.mark.parametrize("m,expect", [(16, True), (256, True), (257, False), (384, False)])
def test_proj_cutover(m, expect):
    x, w = _xw(m, 6144, 4096)
    assert gemm._use_wide(m, 6144, 4096, x, w) is expect


# Llama-3-70B: hidden 8192, so qkv (8192 -> 10240) and o (8192 -> 8192) also have K = 8192; they
# are projections ("proj" cutover), only the narrowing 28672 -> 8192 down projection is "down"
@pytest.mark.parametrize("n,k,m,expect", [
    (10240, 8192, 256, True), (10240, 8192, 257, False), (10240, 8192, 512, False),   # qkv
    (8192, 8192, 256, True), (8192, 8192, 512, True), (8192, 8192, 513, False),      # o (wide_o_max_m)
    (8192, 28672, 384, True), (8192, 28672, 385, False), (8192, 28672, 512, False),   # down
])
def test_70b_roles(n, k, m, expect):
    x, w = _xw(m, n, k)
    assert gemm._use_wide(m, n, k, x, w) is expect


def test_down_role_rule():
    assert gemm.is_down_proj(4096, 14336) and gemm.is_down_proj(8192, 28672)
    assert not gemm.is_down_proj(10240, 8192) and not gemm.is_down_proj(8192, 8192)
    assert not gemm.is_down_proj(4096, 4096) and not gemm.is_down_proj(128256, 4096)


def test_down_cap_can_exceed_512():
    from distributed_llms_amd import knobs
    knobs.update(wide_down_max_m=768)
    x, w = _xw(768, 4096, 14336)
    assert gemm._use_wide(768, 4096, 14336, x, w)
    xg, wg = _xw(768, 2 * 14336, 4096)
    assert not gemm._use_wide(768, wg.shape[0], 4096, xg, wg, swiglu=True)


def test_wide_off_and_dtype_disable_wide():
    from distributed_llms_amd import knobs
    x, w = _xw(128, 4096, 4096)
    assert not gemm._use_wide(128, 4096, 4096, x.float(), w.float())
    knobs.update(wide="none")
    assert not gemm._use_wide(128, 4096, 4096, x, w)


def test_sq_only_on_unsplit_grids():
    """gemm_sq (256 x 256 tiles) serves 225 <= M <= 256 only where its grid needs no K split: the
    LM head and the 70B gate|up (profiles/wide_gemm.md)."""
    from distributed_llms_amd import knobs
    assert gemm.use_sq(256, 128256, 4096) and not gemm.use_sq(192, 128256, 4096)
    assert gemm.use_sq(256, 57344, 8192, swiglu=True)
    assert not gemm.use_sq(128, 128256, 4096)                      # 128-row tile of the wide kernel
    for n, k, sw in ((6144, 4096, False), (4096, 4096, False), (28672, 4096, True), (4096, 14336, False),
                     (10240, 8192, False), (8192, 28672, False), (32000, 4096, False)):
        assert not gemm.use_sq(256, n, k, swiglu=sw), (n, k)
    knobs.update(sq_split=True)
    assert gemm.use_sq(256, 4096, 14336)
    assert gemm.sq_splits(256, 4096, 14336) == 16 and gemm.sq_splits(256, 6144, 4096) == 10


def test_knobs_move_the_cutovers_and_reject_unknown_names():
    from distributed_llms_amd import knobs
    x, w = _xw(384, 6144, 4096)
    assert not gemm._use_wide(384, 6144, 4096, x, w)
    knobs.update(wide_proj_max_m=512)
    assert gemm._use_wide(384, 6144, 4096, x, w)
    knobs.update({"wide": "none"})
    assert not gemm._use_wide(16, 6144, 4096, x, w)
    with pytest.raises(ValueError):
        knobs.update(no_such_knob=1)
    assert knobs.parse("wide_variant=1, defer_qkv=1") == {"wide_variant": "1", "defer_qkv": "1"}
    assert knobs.K.defer_qkv is True and "defer_qkv" not in knobs.changed()      # the shipped default
    knobs.update(knobs.parse('{"defer_qkv": "false"}'))
    assert knobs.K.defer_qkv is False and knobs.changed()["defer_qkv"] is False


def test_prefill_gemms_go_to_hand_written_kernels():
    """Every prefill projection above the decode ranges runs on the persistent schedule-2 kernel
    (gemm_pf): gate|up with the SwiGLU from knobs.pp_swiglu_min_m, qkv / o / down from
    pp_proj_min_m -- hipBLASLt only for shapes none of the kernels takes (N % 256, a bias)."""
    from distributed_llms_amd import knobs
    x, w = _xw(32768, 28672, 4096)
    kn = knobs.K
    assert kn.pp_persistent and kn.pp_swiglu_min_m <= 257 and kn.pp_proj_min_m <= 257
    assert gemm._use_pp(32768, 28672, 4096, x, w, kn.pp_swiglu_min_m)
    assert gemm._use_pp(1024, 28672, 4096, x, w, kn.pp_swiglu_min_m)
    assert gemm._use_pp(32768, 6144, 4096, x, w, kn.pp_proj_min_m)
    assert gemm._use_pp(32768, 4096, 14336, x, w, kn.pp_proj_min_m)
    assert not gemm._use_pp(32768, 28672 + 128, 4096, x, w, kn.pp_swiglu_min_m)   # N % 256
    knobs.update(pp_swiglu_min_m=0)
    assert not gemm._use_pp(32768, 28672, 4096, x, w, knobs.K.pp_swiglu_min_m)


def test_decode_lm_head_goes_to_gemm_pp():
    from distributed_llms_amd import knobs
    x, w = _xw(256, 128256, 4096)
    kn = knobs.K
    assert 0 < kn.pp_head_min_m <= 256 and gemm._use_pp(256, 128256, 4096, x, w, 1)
    assert gemm.PP_HEAD_VARIANT & 64 and gemm.PP_HEAD_VARIANT & 2


def test_wide_splits_leave_comm_cus_free():
    """An RCCL pipeline stage reserves CUs for its spinning comm kernels: every split-K grid then
    fits one workgroup per remaining CU (no second round for the workgroups the comm kernel blocks)."""
    from distributed_llms_amd.ops import gemm
    shapes = [(256, 4096, 14336), (256, 4096, 4096), (256, 6144, 4096), (128, 4096, 4096), (64, 8192, 28672)]
    base = [gemm.wide_splits(*s) for s in shapes]
    gemm.reserve_cus_for_comm(16)
    try:
        for (m, n, k), b in zip(shapes, base):
            s = gemm.wide_splits(m, n, k)
            tiles = (n // 128) * (-(-m // gemm.wide_row_tile(m, n, k)))
            assert tiles * s <= 240 or s == 1, (m, n, k, s)
            assert s <= b
        assert gemm.wide_splits(256, 4096, 14336) == 7
    finally:
        gemm.release_cus_for_comm()
    assert [gemm.wide_splits(*s) for s in shapes] == base


def test_pf_dynamic_auto_follows_comm_reservation():
    from distributed_llms_amd import knobs
    from distributed_llms_amd.ops import gemm
    assert knobs.K.pf_dynamic == "auto" and not gemm.pf_dynamic()
    gemm.reserve_cus_for_comm(16)
    try:
        assert gemm.pf_dynamic()
        with knobs.override(pf_dynamic="off"):
            assert not gemm.pf_dynamic()
    finally:
        gemm.release_cus_for_comm()
    with knobs.override(pf_dynamic=True):
        assert gemm.pf_dynamic()
    with knobs.override(pf_dynamic=0):
        assert not gemm.pf_dynamic()


def test_medium_m_dispatch_follows_the_measured_table():
    """profiles/round5_medium_m_gemm.md: between the decode cutovers and a full gemm_pf grid the
    split-K gemm_pp wins; the o-projection stays on gemm_wide to M = 512, down to M = 384."""
    import torch
    from distributed_llms_amd.ops import gemm
    cpu = torch.device("cpu")
    # gemm_pf only with a full grid: (M / 256) x (N / 256) tiles >= CUs, rounds mostly full
    assert not gemm.pf_fills(2048, 6144, cpu)          # 192 tiles
    assert not gemm.pf_fills(640, 28672, cpu)          # 336 tiles: 2 rounds, 66 % full
    assert gemm.pf_fills(1024, 28672, cpu)             # 448 tiles: 88 % full
    assert gemm.pf_fills(4096, 4096, cpu) and gemm.pf_fills(32768, 6144, cpu)
    assert not gemm.pf_fills(4096, 6144, cpu)          # 384 tiles: 75 % full
    x, w = _xw(512, 4096, 4096)
    assert gemm._use_wide(512, 4096, 4096, x, w)       # o
    x, w = _xw(320, 6144, 4096)
    assert not gemm._use_wide(320, 6144, 4096, x, w)   # qkv -> split-K gemm_pp
    x, w = _xw(384, 4096, 14336)
    assert gemm._use_wide(384, 4096, 14336, x, w)      # down
    x, w = _xw(512, 4096, 14336)
    assert not gemm._use_wide(512, 4096, 14336, x, w)


def test_decode_gate_up_on_gemm_pp_128_column_tile():
    """knobs.pp_gate_up_min_m: the 8B gate|up at 200 <= M <= 256 runs on gemm_pp's 128-column tile
    with nontemporal weights (224 tiles: one round), the 70B gate|up on its 256-column tile (224
    tiles); not below the cutover, not while comm kernels reserve CUs."""
    from distributed_llms_amd.ops import gemm
    calls = []
    orig_pp, orig_wide, orig_sq = gemm.linear_pp, gemm.linear_wide, gemm.linear_sq
    gemm.linear_pp = lambda *a, **k: calls.append(("pp", k.get("variant"), k.get("splits")))
    gemm.linear_wide = lambda *a, **k: calls.append(("wide",))
    gemm.linear_sq = lambda *a, **k: calls.append(("sq",))
    try:
        gemm.linear_swiglu(*_xw(256, 28672, 4096))
        gemm.linear_swiglu(*_xw(192, 28672, 4096))
        gemm.linear_swiglu(*_xw(256, 57344, 8192))
        gemm.reserve_cus_for_comm(16)
        try:
            gemm.linear_swiglu(*_xw(256, 28672, 4096))
        finally:
            gemm.release_cus_for_comm()
    finally:
        gemm.linear_pp, gemm.linear_wide, gemm.linear_sq = orig_pp, orig_wide, orig_sq
    assert calls[0] == ("pp", gemm.PP_GATE_UP_VARIANT, 1)
    assert calls[1][0] == "wide" and calls[3][0] == "wide"
    assert calls[2] == ("pp", gemm.PP_GATE_UP_VARIANT & ~1, 1)       # 70B: 224 x 256-column tiles


def test_long_k_down_on_split_gemm_pp():
    """knobs.pp_down_min_k: the 70B down projection (K = 28672) at decode M on split gemm_pp
    128-column tiles (64 tiles x 4 slices, nontemporal weights); the 8B down (K = 14336) and other
    projections keep gemm_wide."""
    from distributed_llms_amd.ops import gemm
    calls = []
    orig_pp, orig_wide = gemm.linear_pp, gemm.linear_wide
    gemm.linear_pp = lambda *a, **k: calls.append(("pp", k.get("splits"), k.get("variant")))
    gemm.linear_wide = lambda *a, **k: calls.append(("wide",))
    try:
        gemm.linear(*_xw(256, 8192, 28672), defer=True)
        gemm.linear(*_xw(256, 4096, 14336), defer=True)
        gemm.linear(*_xw(128, 8192, 28672), defer=True)
    finally:
        gemm.linear_pp, gemm.linear_wide = orig_pp, orig_wide
    assert calls == [("pp", 4, 64 | 2 | 1), ("wide",), ("wide",)]


def test_o_projection_runs_as_two_128_row_tiles_at_decode():
    """knobs.wide_small_bm = 128 (default): the 8B o-projection (N K <= 4096^2) at M = 256 runs as
    2 x 128-row tiles x 4 K slices (engine +0.75 %); qkv, the down projection and the SwiGLU keep
    the 256-row tile."""
    from distributed_llms_amd.ops import gemm
    assert gemm.wide_row_tile(256, 4096, 4096) == 128
    assert gemm.wide_splits(256, 4096, 4096) == 4
    assert gemm.wide_row_tile(256, 6144, 4096) == 256
    assert gemm.wide_row_tile(256, 4096, 14336) == 256
    assert gemm.wide_row_tile(256, 28672, 4096, swiglu=True) == 256
    assert gemm.wide_row_tile(64, 4096, 4096) == 64


def test_lm_head_leaves_gemm_pp_while_comm_cus_are_reserved():
    from distributed_llms_amd.ops import gemm
    x, w = _xw(256, 128256, 4096)
    assert gemm._use_pp(256, 128256, 4096, x, w, 1)
    calls = []
    orig_pp, orig_wide = gemm.linear_pp, gemm.linear_wide
    gemm.linear_pp = lambda *a, **k: calls.append("pp")
    gemm.linear_wide = lambda *a, **k: calls.append("wide")
    try:
        gemm.linear(x, w)
        gemm.reserve_cus_for_comm(16)
        gemm.linear(x, w)
    finally:
        gemm.release_cus_for_comm()
        gemm.linear_pp, gemm.linear_wide = orig_pp, orig_wide
    assert calls == ["pp", "wide"]


def test_prefill_rope_in_attention_gated_on_block_table_width():
    """Advisor round 5: block tables wider than the LDS prefill kernel stages (sequences past 32k
    tokens) must take the write_q=True append + plain prefill kernel, not the in-kernel q-RoPE."""
    from distributed_llms_amd import knobs, ops
    with knobs.override(prefill_attn=4, prefill_fused_rope=True):
        assert ops.prefill_rope_in_attention()
        assert ops.prefill_rope_in_attention(ops.PF_MAX_CHUNKS)
        assert not ops.prefill_rope_in_attention(ops.PF_MAX_CHUNKS + 1)
    with knobs.override(prefill_attn=3, prefill_fused_rope=True):
        assert not ops.prefill_rope_in_attention(16)


def test_prefill_attention_auto_version():
    """knobs.prefill_attn = 0 (default): the persistent 32x32x16 kernel (9) from prefill_w32_min_q
    query rows at head_dim 128, its one-shot form (7) while comm kernels reserve CUs, v4 for short
    prompts and for head_dim 64; an explicit knob wins.  Every auto choice takes the in-kernel q-RoPE."""
    from distributed_llms_amd import knobs, ops
    from distributed_llms_amd.ops import gemm
    with knobs.override(prefill_attn=0, prefill_w32_min_q=512, prefill_fused_rope=True):
        assert ops.prefill_attn_version(128, 128) == 4
        assert ops.prefill_attn_version(511, 128) == 4
        assert ops.prefill_attn_version(512, 128) == 9
        assert ops.prefill_attn_version(16384, 128) == 9
        assert ops.prefill_attn_version(4096, 64) == 4
        assert ops.prefill_rope_in_attention(64)
        gemm.reserve_cus_for_comm(16)
        try:
            assert ops.prefill_attn_version(4096, 128) == 7
        finally:
            gemm.release_cus_for_comm()
        assert ops.prefill_attn_version(4096, 128) == 9
    for v in (3, 4, 6, 7, 9):
        with knobs.override(prefill_attn=v):
            assert ops.prefill_attn_version(4096, 128) == v
