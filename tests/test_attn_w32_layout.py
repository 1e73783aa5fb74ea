"""CPU check of the index algebra of the 32x32x16-MFMA prefill attention (attention.hip,
attn_prefill_w32_kernel, prefill versions 6 / 7): a numpy model of v_mfma_f32_32x32x16_bf16's operand
and result layouts, fed exactly as the kernel feeds it -- K rows at w32_krow(m) of the krow32-permuted
cache block, the P.V B operand taken straight from 8 consecutive score registers, the V^T A operand
read from key group 2 h + hi of the [4][D][8] V^T block -- reproduces softmax(Q K^T) V of one tile.
A wrong permutation here would show up on the GPU only as slightly-off attention rows."""
import numpy as np


def krow32(j):          # common.h: K row of key j in a 32-key block
    return ((j & 4) << 2) + ((j >> 3) << 2) + (j & 3)


def w32_krow(m):        # attention.hip: physical K row the QK^T A operand reads for MFMA row m
    return (((m >> 3) & 1) << 4) | ((m >> 4) << 3) | (((m >> 2) & 1) << 2) | (m & 3)


def mfma_32x32x16(a_lanes, b_lanes, c_lanes):
    """a_lanes / b_lanes: [64][8] per-lane operands, c_lanes: [64][16] accumulators.
    A[i][k]: lane i % 32 + 32 (k // 8), element k % 8;  B[k][j]: lane j + 32 (k // 8), element k % 8;
    D[i][j]: lane j + 32 ((i // 4) % 2), register 4 (i // 8) + i % 4."""
    A = np.zeros((32, 16))
    B = np.zeros((16, 32))
    for lane in range(64):
        for e in range(8):
            A[lane % 32][8 * (lane // 32) + e] = a_lanes[lane][e]
            B[8 * (lane // 32) + e][lane % 32] = b_lanes[lane][e]
    D = A @ B
    out = [list(c) for c in c_lanes]
    for lane in range(64):
        for r in range(16):
            i = 8 * (r // 4) + 4 * (lane // 32) + r % 4
            out[lane][r] += D[i][lane % 32]
    return out


def test_w32_krow_is_krow32_of_the_bit_swapped_key():
    for m in range(32):
        pi = (m & ~0b1100) | ((m >> 2) & 1) << 3 | ((m >> 3) & 1) << 2
        assert w32_krow(m) == krow32(pi)
    assert sorted(w32_krow(m) for m in range(32)) == list(range(32))


def test_w32_reads_are_bank_conflict_free():
    """ds_read_b128 services lanes in 4 groups of 16; K rows are XOR-swizzled by row & 15 and the V^T
    fragment of lane m is dim 32 dt + m: every group must hit 16 distinct 16-byte slots."""
    groups = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
    for grp in groups:
        for ks in range(8):
            for hi in range(2):
                slots = {((2 * ks + hi) ^ (w32_krow(m) & 15)) for m in grp}
                assert len(slots) == 16
        for dt in range(4):
            assert len({(32 * dt + m) % 16 for m in grp}) == 16


def test_w32_tile_reproduces_attention():
    rng = np.random.default_rng(0)
    D = 128
    q = rng.standard_normal((32, D))              # 32 columns (8 rows x 4 heads); one kv head
    keys = rng.standard_normal((64, D))           # a 64-key tile: blocks 0 and 1
    vals = rng.standard_normal((64, D))
    # the paged cache's block images: K rows permuted by krow32, V^T as [4 groups][D][8 keys]
    kblk = [np.zeros((32, D)) for _ in range(2)]
    vt = [np.zeros((4, D, 8)) for _ in range(2)]
    for b in range(2):
        for j in range(32):
            kblk[b][krow32(j)] = keys[32 * b + j]
            vt[b][j // 8, :, j % 8] = vals[32 * b + j]
    bf = lambda x: x                              # noqa: E731  (exact arithmetic for the layout check)
    # S^T = K Q^T, per block: 8 k-slices of 16 dims
    s = []
    for b in range(2):
        acc = [[0.0] * 16 for _ in range(64)]
        for ks in range(8):
            a = [kblk[b][w32_krow(l % 32)][16 * ks + 8 * (l // 32): 16 * ks + 8 * (l // 32) + 8] for l in range(64)]
            bq = [q[l % 32][16 * ks + 8 * (l // 32): 16 * ks + 8 * (l // 32) + 8] for l in range(64)]
            acc = mfma_32x32x16(a, bq, acc)
        s.append(acc)
    # the kernel's claim: register r of block b, lane l, is the score of key 32 b + 16 (r >> 3) + 8 hi + (r & 7)
    full = q @ keys.T                             # [col][key]
    for b in range(2):
        for l in range(64):
            hi = l // 32
            for r in range(16):
                key = 32 * b + 16 * (r >> 3) + 8 * hi + (r & 7)
                assert np.isclose(s[b][l][r], full[l % 32][key])
    # softmax in-lane (max over both halves of the column), P.V from the score registers
    p = [[np.exp(np.array(s[b][l]) - full[l % 32].max()) for l in range(64)] for b in range(2)]
    o = [[[0.0] * 16 for _ in range(64)] for _ in range(D // 32)]
    for dt in range(D // 32):
        for bh in range(4):
            b, h = bh >> 1, bh & 1
            va = [vt[b][2 * h + l // 32, 32 * dt + l % 32, :] for l in range(64)]
            pb = [bf(p[b][l][8 * h: 8 * h + 8]) for l in range(64)]
            o[dt] = mfma_32x32x16(va, pb, o[dt])
    ref = np.exp(full - full.max(axis=1, keepdims=True)) @ vals      # [col][d], unnormalized
    for dt in range(D // 32):
        for l in range(64):
            for r in range(16):
                d = 32 * dt + 8 * (r // 4) + 4 * (l // 32) + r % 4   # the output image's dim for acc[dt][r]
                assert np.isclose(o[dt][l][r], ref[l % 32][d])
