"""HIP kernel numerics vs the plain-PyTorch fp32 reference of the same op (gfx950 only)."""
import math

import pytest
import torch

from distributed_llms_amd import _ext, ops
from distributed_llms_amd.ops import reference as ref

pytestmark = pytest.mark.gpu


def _bf(*shape, scale=1.0, dev="cuda"):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def test_native_module_loaded(cuda):
    k = _ext.kernels()
    assert k.arch == "gfx950"


@pytest.mark.parametrize("rows,hidden", [(1, 4096), (7, 4096), (64, 8192), (3, 768), (5, 128)])
def test_rms_norm(cuda, rows, hidden):
    x, w = _bf(rows, hidden), _bf(hidden)
    y = ops.rms_norm(x, w, 1e-5)
    yr = ref.rms_norm(x.float(), w.float(), 1e-5)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("rows,hidden", [(1, 4096), (33, 4096), (16, 8192)])
def test_fused_add_rms_norm(cuda, rows, hidden):
    x, r, w = _bf(rows, hidden), _bf(rows, hidden), _bf(hidden)
    r0 = r.clone()
    y, r2 = ops.fused_add_rms_norm(x, r, w, 1e-5)
    rr = (x.float() + r0.float()).to(torch.bfloat16)
    torch.testing.assert_close(r2, rr, atol=0, rtol=0)
    yr = ref.rms_norm(rr.float(), w.float(), 1e-5)
    torch.testing.assert_close(y.float(), yr, atol=2e-2, rtol=2e-2)


def test_embedding(cuda):
    table = _bf(1000, 512)
    ids = torch.randint(0, 1000, (37,), device="cuda", dtype=torch.int32)
    torch.testing.assert_close(ops.embedding(ids, table), table[ids.long()], atol=0, rtol=0)


def test_silu_mul(cuda):
    gu = _bf(19, 2 * 1024)
    torch.testing.assert_close(ops.silu_mul(gu).float(), ref.silu_mul(gu.float()), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("rows,vocab", [(1, 128256), (9, 50257), (4, 32000)])
def test_argmax(cuda, rows, vocab):
    logits = _bf(rows, vocab, scale=3.0)
    expect = logits.float().argmax(-1).to(torch.int32)
    torch.testing.assert_close(ops.argmax(logits), expect)


@pytest.mark.parametrize("rows,vocab", [(256, 128256), (3, 50257)])
def test_argmax_ties_take_the_first_index(cuda, rows, vocab):
    """Coarse logits (many equal maxima per row, spread over every thread's strided scan), an
    all-equal row and a row whose maximum sits in the ragged tail: the first maximal index, as torch."""
    logits = (_bf(rows, vocab, scale=3.0).float().round()).to(torch.bfloat16)
    logits[0] = 1.0
    logits[-1, :] = -5.0
    logits[-1, vocab - 3:] = 7.0
    expect = logits.float().argmax(-1).to(torch.int32)
    torch.testing.assert_close(ops.argmax(logits), expect)


def _cache(nb, hkv, d, bs=32):
    k = torch.zeros(nb, hkv, bs, d, dtype=torch.bfloat16, device="cuda")
    v = torch.zeros(nb, hkv, d, bs, dtype=torch.bfloat16, device="cuda")
    return k, v


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (12, 12, 64), (64, 8, 128)])
def test_rope_cache_append(cuda, hq, hkv, d):
    t, nb = 21, 8
    qkv = _bf(t, (hq + 2 * hkv) * d)
    pos = torch.randint(0, 500, (t,), device="cuda", dtype=torch.int32)
    slots = torch.randperm(nb * 32, device="cuda")[:t].to(torch.int32)
    cs = ref.rope_cos_sin(d, 1024, 500000.0, device="cuda")
    k1, v1 = _cache(nb, hkv, d)
    k2, v2 = _cache(nb, hkv, d)
    q1 = ops.rope_cache_append(qkv, pos, cs, k1, v1, slots, hq, hkv, d)
    q2 = ref.rope_cache_append(qkv.float(), pos, cs, k2, v2, slots, hq, hkv, d)
    torch.testing.assert_close(q1.float(), q2.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(k1.float(), k2.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(v1, v2, atol=0, rtol=0)


@pytest.mark.parametrize("grouped", [True, False])
def test_rope_cache_append_prefill_groups(cuda, grouped):
    """Prefill slot patterns for the grouped V append: aligned whole groups (16-byte stores),
    prompts starting / ending mid-group, a sequence resuming mid-block, non-consecutive slots, a
    ragged tail -- all bit-identical to the reference scatter."""
    from distributed_llms_amd import knobs
    hq, hkv, d, nb = 32, 8, 128, 24
    runs = [(0, 45), (3 * 32, 32), (5 * 32 + 5, 19), (7 * 32 + 8, 3), (9 * 32, 64)]
    sl = [s + i for s, n in runs for i in range(n)] + [20 * 32 + 31, 21 * 32 + 2, 22 * 32 + 9]
    t = len(sl)
    slots = torch.tensor(sl, dtype=torch.int32, device="cuda")
    qkv = _bf(t, (hq + 2 * hkv) * d)
    pos = torch.arange(t, device="cuda", dtype=torch.int32)
    cs = ref.rope_cos_sin(d, 1024, 500000.0, device="cuda")
    k1, v1 = _cache(nb, hkv, d)
    k2, v2 = _cache(nb, hkv, d)
    with knobs.override(v_group_append=grouped):
        assert ops.rope_cache_append(qkv, pos, cs, k1, v1, slots, hq, hkv, d, write_q=False) is None
    ref.rope_cache_append(qkv.float(), pos, cs, k2, v2, slots, hq, hkv, d)
    torch.testing.assert_close(k1.float(), k2.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(v1, v2, atol=0, rtol=0)


def _fill_paged(seq_lens, hkv, d, nb_total=None):
    bs = 32
    nblocks = [(n + bs - 1) // bs for n in seq_lens]
    nb_total = nb_total or sum(nblocks) + 3
    k, v = _cache(nb_total, hkv, d)
    k.normal_()
    v.normal_()
    perm = torch.randperm(nb_total).tolist()
    mb = max(nblocks)
    bt = torch.zeros(len(seq_lens), mb, dtype=torch.int32)
    i = 0
    for s, n in enumerate(nblocks):
        bt[s, :n] = torch.tensor(perm[i:i + n])
        i += n
    return k, v, bt.cuda()


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (64, 8, 128), (12, 12, 64), (4, 1, 128)])
@pytest.mark.parametrize("lens", [[1], [7, 33, 100], [640, 5, 2049, 32]])
def test_paged_attention_decode(cuda, hq, hkv, d, lens):
    k, v, bt = _fill_paged(lens, hkv, d)
    sl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    q = _bf(len(lens), hq, d)
    scale = 1 / math.sqrt(d)
    out = ops.paged_attention_decode(q, k, v, bt, sl, scale)
    expect = ref.paged_attention_decode(q.float(), k.float(), v.float(), bt, sl, scale)
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (12, 12, 64), (4, 1, 128)])
@pytest.mark.parametrize("lens", [[1], [7, 33, 100], [640, 5, 2049, 32]])
@pytest.mark.parametrize("rope", [True, False])
def test_paged_attention_decode_fused_rope(cuda, hq, hkv, d, lens, rope):
    """RoPE + KV append fused into decode attention == rope_cache_append + paged_attention_decode
    (fp32 reference), including what lands in the cache; also with split-KV (long contexts)."""
    k, v, bt = _fill_paged(lens, hkv, d)
    b = len(lens)
    sl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    pos = sl - 1
    # slot of the new token: position len-1 inside its sequence's block table
    slots = torch.stack([bt[i, (n - 1) // 32] * 32 + (n - 1) % 32 for i, n in enumerate(lens)]).to(torch.int32)
    qkv = _bf(b, (hq + 2 * hkv) * d)
    cs = ref.rope_cos_sin(d, 4096, 500000.0, device="cuda") if rope else None
    scale = 1 / math.sqrt(d)
    k1, v1 = k.clone(), v.clone()
    out = ops.paged_attention_decode_rope(qkv, pos, cs, k1, v1, slots, bt, sl, hq, hkv, d, scale)
    k2, v2 = k.float(), v.float()
    q2 = ref.rope_cache_append(qkv.float(), pos, cs, k2, v2, slots, hq, hkv, d)
    expect = ref.paged_attention_decode(q2, k2, v2, bt, sl, scale)
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(k1.float(), k2, atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(v1.float(), v2, atol=0, rtol=0)


@pytest.mark.parametrize("version", ["3", "4", "6", "7", "9"])
@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (64, 8, 128), (12, 12, 64), (8, 4, 64), (16, 16, 128),
                                      (32, 2, 128)])
def test_paged_attention_prefill(cuda, hq, hkv, d, version):
    ctx = [37, 128, 300, 5]
    qlen = [37, 64, 1, 5]       # second/third: chunked prefill with prior context
    k, v, bt = _fill_paged(ctx, hkv, d)
    cu = torch.tensor([0] + list(torch.tensor(qlen).cumsum(0)), dtype=torch.int32, device="cuda")
    sl = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    q = _bf(sum(qlen), hq, d)
    scale = 1 / math.sqrt(d)
    out = ops.paged_attention_prefill(q, k, v, bt, cu, sl, scale, version=int(version))
    expect = ref.paged_attention_prefill(q.float(), k.float(), v.float(), bt, cu, sl, scale)
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("version", ["3", "4", "6", "7", "9"])
def test_paged_attention_prefill_long(cuda, version):
    """Long prompts: > 64 KV chunks per sequence (block-id reloads), many workgroups per
    (sequence, kv head), a chunked prefill that starts mid-block."""
    hq, hkv, d = 32, 8, 128
    ctx = [2300, 777, 64]
    qlen = [900, 777, 33]
    k, v, bt = _fill_paged(ctx, hkv, d)
    cu = torch.tensor([0] + list(torch.tensor(qlen).cumsum(0)), dtype=torch.int32, device="cuda")
    sl = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    q = _bf(sum(qlen), hq, d)
    scale = 1 / math.sqrt(d)
    out = ops.paged_attention_prefill(q, k, v, bt, cu, sl, scale, version=int(version))
    expect = ref.paged_attention_prefill(q.float(), k.float(), v.float(), bt, cu, sl, scale)
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("version", ["4", "7", "9"])
def test_paged_attention_prefill_many_short(cuda, version):
    """Many short prompts (a few with prior context): 512 (sequence, kv head) groups of one- and
    two-tile row blocks -- the persistent kernel (9) walks several per workgroup, switching items
    every tile or two."""
    hq, hkv, d = 32, 8, 128
    g = torch.Generator().manual_seed(3)
    qlen = [int(x) for x in torch.randint(1, 200, (64,), generator=g)]
    ctx = [q + (40 if i % 7 == 0 else 0) for i, q in enumerate(qlen)]
    k, v, bt = _fill_paged(ctx, hkv, d)
    cu = torch.tensor([0] + list(torch.tensor(qlen).cumsum(0)), dtype=torch.int32, device="cuda")
    sl = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    q = _bf(sum(qlen), hq, d)
    scale = 1 / math.sqrt(d)
    out = ops.paged_attention_prefill(q, k, v, bt, cu, sl, scale, version=int(version))
    expect = ref.paged_attention_prefill(q.float(), k.float(), v.float(), bt, cu, sl, scale)
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)


def test_attention_masked_spike(cuda):
    """Force the online-softmax rescale: one key far above the rest, late in the sequence."""
    hq, hkv, d = 32, 8, 128
    lens = [1000]
    k, v, bt = _fill_paged(lens, hkv, d)
    q = _bf(1, hq, d)
    blk = bt[0, 900 // 32].item()
    k[blk, :, 900 % 32, :] = q[0, ::4].to(k.dtype) * 4
    sl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    out = ops.paged_attention_decode(q, k, v, bt, sl, 1 / math.sqrt(d))
    expect = ref.paged_attention_decode(q.float(), k.float(), v.float(), bt, sl, 1 / math.sqrt(d))
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("splits", [3, 5, 6])
@pytest.mark.parametrize("b", [100, 256])
def test_decode_rope_consumes_splitk_qkv_bit_exact(cuda, b, splits):
    """The fused decode kernel summing the qkv projection's f32 split-K slabs itself gives exactly
    the result of reducing first (same slab order, same bf16 rounding)."""
    from distributed_llms_amd.ops import gemm
    hq, hkv, d, hidden = 32, 8, 128, 4096
    lens = [int(x) for x in torch.randint(40, 300, (b,))]
    k, v, bt = _fill_paged(lens, hkv, d)
    x = _bf(b, hidden)
    w = _bf((hq + 2 * hkv) * d, hidden, scale=0.02)
    sl = torch.tensor(lens, dtype=torch.int32, device="cuda")
    pos = sl - 1
    slots = torch.stack([bt[i, (lens[i] - 1) // 32] * 32 + (lens[i] - 1) % 32 for i in range(b)]).to(torch.int32)
    cs = ref.rope_cos_sin(d, 4096, 500000.0, device="cuda")
    part = gemm.linear_wide(x, w, splits=splits, defer=True)
    assert isinstance(part, gemm.SplitKPartial)
    k1, v1, k2, v2 = k.clone(), v.clone(), k.clone(), v.clone()
    o1 = ops.paged_attention_decode_rope(part, pos, cs, k1, v1, slots, bt, sl, hq, hkv, d, 1 / math.sqrt(d))
    qkv = part.materialize()
    o2 = ops.paged_attention_decode_rope(qkv, pos, cs, k2, v2, slots, bt, sl, hq, hkv, d, 1 / math.sqrt(d))
    torch.testing.assert_close(o1, o2, atol=0, rtol=0)
    torch.testing.assert_close(k1, k2, atol=0, rtol=0)
    torch.testing.assert_close(v1, v2, atol=0, rtol=0)


@pytest.mark.parametrize("version", [4, 6, 7, 9])
@pytest.mark.parametrize("hq,hkv,d", [(32, 8, 128), (8, 4, 64)])
def test_prefill_attention_with_q_rope_in_kernel(cuda, hq, hkv, d, version):
    """knobs.prefill_fused_rope: rope_cache_append(write_q=False) appends K / V only and the LDS prefill
    kernel rotates q from the raw qkv projection in registers.  Same cache contents, and the attention
    output matches the two-pass form (rotated q written, then attended) and the fp32 reference."""
    from distributed_llms_amd import knobs
    ctx = [37, 128, 300, 5]
    qlen = [37, 64, 1, 5]
    t = sum(qlen)
    k1, v1, bt = _fill_paged(ctx, hkv, d)
    k2, v2 = k1.clone(), v1.clone()
    cu = torch.tensor([0] + list(torch.tensor(qlen).cumsum(0)), dtype=torch.int32, device="cuda")
    sl = torch.tensor(ctx, dtype=torch.int32, device="cuda")
    pos = torch.cat([torch.arange(c - q, c) for c, q in zip(ctx, qlen)]).to(torch.int32).cuda()
    # the new tokens' slots: the positions' places in each sequence's blocks
    btc = bt.cpu()
    slots = torch.tensor([int(btc[i, p // 32]) * 32 + p % 32 for i, (c, q) in enumerate(zip(ctx, qlen))
                          for p in range(c - q, c)], dtype=torch.int32, device="cuda")
    qkv = _bf(t, (hq + 2 * hkv) * d)
    cs = ref.rope_cos_sin(d, 1024, 500000.0, device="cuda")
    scale = 1 / math.sqrt(d)
    with knobs.override(prefill_attn=version, prefill_fused_rope=True):
        q = ops.rope_cache_append(qkv, pos, cs, k1, v1, slots, hq, hkv, d)
        two_pass = ops.paged_attention_prefill(q, k1, v1, bt, cu, sl, scale)
        assert ops.rope_cache_append(qkv, pos, cs, k2, v2, slots, hq, hkv, d, write_q=False) is None
        fused = ops.paged_attention_prefill_rope(qkv, pos, cs, k2, v2, bt, cu, sl, hq, d, scale, max_q_len=max(qlen))
    assert torch.equal(k1, k2) and torch.equal(v1, v2)
    torch.testing.assert_close(fused.float(), two_pass.float(), atol=4e-3, rtol=4e-3)
    expect = ref.paged_attention_prefill(ref.rope_q(qkv.float(), pos, cs, hq, d), k1.float(), v1.float(), bt, cu,
                                         sl, scale)
    torch.testing.assert_close(fused.float(), expect, atol=2e-2, rtol=2e-2)
