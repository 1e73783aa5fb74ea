// K6 + K7: paged attention on MFMA (v_mfma_f32_16x16x32_bf16), decode and prefill.
//
// Layout (one pair per layer, block_size BS = 32 tokens):
//   k_cache [NB, Hkv, 32, D]   key rows contiguous       -> QK A-operand = 16 B / lane
//   v_cache [NB, Hkv, D, 32]   V stored transposed       -> PV A-operand = 2 x 8 B / lane
// The 16 MFMA columns are (query row, head-in-GQA-group) pairs, so the K/V bytes of
// one kv-head are read once for all G = Hq/Hkv query heads:
//   decode : 1 query  x G heads   (G <= 16 columns used)
//   prefill: 16/G rows x G heads  (all 16 columns used when G | 16)
// Scores are computed transposed (S^T = K Q^T): each lane then holds 8 keys of ONE
// column, the row max needs 2 cross-lane shuffles, and the lane's 8 probabilities are
// exactly its B-operand fragment for O^T += V^T P^T (the k-order of the PV product is
// permuted to match, so P never leaves the lane).  Online softmax in base 2.
#include "common.h"
#include "launchers.h"


namespace dllm {

constexpr int kBS = 32;       // tokens per KV block (== keys per MFMA chunk)
#ifndef DLLM_VFULL
#define DLLM_VFULL 1
#endif
// fused decode appends v by rewriting its key group's whole V^T tile (see patch() below)
constexpr bool kVFullLines = DLLM_VFULL;
constexpr int kWaves = 4;     // waves per workgroup
typedef __attribute__((address_space(3))) void* lds_vptr_a;
typedef __attribute__((address_space(1))) void* glb_vptr_a;

template <int D>
struct WaveState {
  f32x4 acc[D / 16];
  float m;      // running max (log2 domain) of this lane's column
  float lsum;   // lane-partial softmax denominator
};

// One 32-key chunk's operands, loaded into registers: K rows as two 16-key A tiles (physical
// rows, see krow32 in common.h), V^T as the A fragments of the P.V MFMA (keys 8g..8g+7 of
// lane group g: one 16-byte load from the [4][D][8] V^T block).
template <int D>
struct KVChunk {
  bf16x8 ka[D / 32], kb[D / 32];
  bf16x8 v[D / 16];
};

template <int D, bool NT = false>
__device__ __forceinline__ void load_chunk(KVChunk<D>& c, const bf16* __restrict__ kblk,
                                           const bf16* __restrict__ vblk, int lane) {
  const int r = lane & 15, g = lane >> 4;
// NT: the decode wave reads each K/V line once per step (cold, HBM): nontemporal loads cut the
// attention alone 41.4 -> 35.3 us at B=256 / ctx 192 (profiles/attn_fused_ablation.md); prefill
// re-reads a sequence's K/V for every q tile and keeps the default policy
#define DLLM_KVLD(p) (NT ? __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p)) \
                         : *reinterpret_cast<const bf16x8*>(p))
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    c.ka[ks] = DLLM_KVLD(kblk + r * D + ks * 32 + 8 * g);
    c.kb[ks] = DLLM_KVLD(kblk + (16 + r) * D + ks * 32 + 8 * g);
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    c.v[dt] = DLLM_KVLD(vblk + g * 8 * D + (dt * 16 + r) * 8);
#undef DLLM_KVLD
}

// Online-softmax update of the wave's 16 columns with one loaded chunk.
//   kmax_col : last admissible key index for this lane's column (causal / range), inclusive
//   MASK     : false when the caller knows every key of the chunk is admissible for every column
//              (prefill chunks strictly below the diagonal): no per-score compare / select
// VALU economy (long prefill is VALU-bound: ~330 VALU per 32 MFMAs, MFMA 25 % busy --
// profiles/round5_prefill_attn_valu.md): the running max is taken on the raw scores and scaled
// once (x -> x * scale is monotonic, so the max is the same number), the scale folds into the
// exponent's FMA, and exp2 is the bare v_exp_f32 (libm's exp2f adds a denormal-range fix-up of
// four instructions per call; results below 2^-126 of the row max flush to zero), and the
// accumulator rescale is skipped when no column's max moved.
template <int D, bool MASK = true>
__device__ __forceinline__ void compute_chunk(WaveState<D>& st, const bf16x8 (&qf)[D / 32], const KVChunk<D>& c,
                                              int t0, int kmax_col, float scale_log2, int lane) {
  const int g = lane >> 4;
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < D / 32; ++ks) {
    s0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c.ka[ks], qf[ks], s0, 0, 0, 0);
    s1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(c.kb[ks], qf[ks], s1, 0, 0, 0);
  }
  float p[8];
  float cm = -INFINITY;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (MASK) {
      const int k0 = t0 + 8 * g + i, k1 = t0 + 8 * g + 4 + i;   // S^T rows 4g+i / 16+4g+i (krow32)
      p[i] = (k0 <= kmax_col) ? s0[i] : -INFINITY;
      p[4 + i] = (k1 <= kmax_col) ? s1[i] : -INFINITY;
    } else {
      p[i] = s0[i];
      p[4 + i] = s1[i];
    }
    cm = fmaxf(cm, fmaxf(p[i], p[4 + i]));
  }
  cm = rows_max(cm);                                // VALU row swaps, no LDS round trip
  cm *= scale_log2;
  // No early exit here: MFMA reads all 64 lanes' operands regardless of EXEC, so every
  // lane must run the same instruction stream. A fully masked column uses mref = 0,
  // which turns its probabilities (and its alpha) into exact zeros.
  const float mn = fmaxf(st.m, cm);
  const float mref = (mn == -INFINITY) ? 0.f : mn;
  const float alpha = __builtin_amdgcn_exp2f(st.m - mref);
  st.m = mn;
  // exponent arguments two per v_pk_fma_f32 (the same fused multiply-add per element), the
  // probabilities summed as a pairwise tree on v_pk_add_f32: 4 + 4 VALU where scalar code takes 8 + 8
  bf16x8 pb;
  f32x2 e2[4];
  const f32x2 sc2 = {scale_log2, scale_log2}, mr2 = {-mref, -mref};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x2 x = __builtin_elementwise_fma(f32x2{p[2 * j], p[2 * j + 1]}, sc2, mr2);
    e2[j] = f32x2{__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
    pb[2 * j] = f2bf(e2[j][0]);
    pb[2 * j + 1] = f2bf(e2[j][1]);
  }
  const f32x2 s2 = (e2[0] + e2[1]) + (e2[2] + e2[3]);
  st.lsum = st.lsum * alpha + (s2[0] + s2[1]);
  // alpha is exactly 1 wherever the running max did not move (exp2(0)), the common case once a
  // row's max has settled: skip the accumulator rescale when that holds for the whole wave (bit-exact)
  if (__any(alpha != 1.f)) {
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) st.acc[dt] *= alpha;
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    const bf16x8 va = c.v[dt];
    st.acc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pb, st.acc[dt], 0, 0, 0);
  }
}

template <int D>
__device__ __forceinline__ void init_state(WaveState<D>& st) {
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) st.acc[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  st.m = -INFINITY;
  st.lsum = 0.f;
}

// ---------------------------------------------------------------------------
// Decode: grid (num_splits, Hkv / WPB, B), WPB waves per workgroup, ONE wave per
// (split, kv-head, sequence).  The wave walks its split's chunks with a depth-2 software
// pipeline -- chunk c+1's K/V loads are in flight while chunk c's MFMAs and softmax run --
// and the chunk -> block ids come from one lane-parallel load of the block-table row
// (read back with readlane), so the only dependent HBM latency per chunk is the KV
// stream itself.  No LDS, no barrier.  num_splits > 1 writes (o, m, l) partials for the
// split-reduce kernel below.  (The first version used 4 waves per (split, head, seq) with
// chunks round-robin, no cross-chunk prefetch and an LDS combine: 47 us per layer at
// B=256 / ctx 128-256 on Llama-3-8B, profiles/llama3_8b_b256_kernels_auto.md.)
// ---------------------------------------------------------------------------
// Fused RoPE + KV append (decode only): the wave reads its q heads and the new token's k / v
// straight from the qkv projection, rotates q and k in registers (pair (e, e + D/2) lives in
// fragments ks and ks + D/64 of the same lane), writes k and v^T into the paged cache (the
// split that owns key ctx-1 only), and folds the new key in as a one-key register chunk --
// the separate rope_cache_kernel launch and the q round trip disappear.
struct RopeArgs {
  const bf16* qkv;          // [B, (hq + 2 hkv) * D]
  const int32_t* positions; // [B]
  const float* cos_sin;     // [max_pos, D] (first half cos, second half sin) or null (no RoPE)
  const int32_t* slots;     // [B] cache slot of the new token
  // optional: the qkv projection as S split-K partial slabs (common.h part_t) [S][B][(hq + 2 hkv) * D] (qkv
  // unused); summed in slab order and rounded to bf16 -- bit-identical to splitk_reduce + bf16
  const float* part = nullptr;
  int nparts = 0;
  long slab = 0;
};

// 8 consecutive qkv elements starting at row offset `off` of sequence b (bf16 or summed partials).
// NP (0 = bf16 qkv, > 0 = that many slabs, -1 = runtime count) is a compile-time choice: a runtime
// branch here split the kernel's prologue into blocks
// with vmcnt(0) waits at every merge (cold B=256: 48 us vs 40 us without the fused part).
template <int NP>
__device__ __forceinline__ bf16x8 qkv_load8(const RopeArgs& ra, int b, int width, int off) {
  if constexpr (NP == 0) return *reinterpret_cast<const bf16x8*>(ra.qkv + (size_t)b * width + off);
  const size_t p = (size_t)b * width + off;
  f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  if constexpr (NP > 0) {
    // compile-time slab count: all 2 * NP loads in flight before the first add (a runtime loop
    // waits on each slab in turn: NP dependent round trips in front of the KV stream)
    f32x4 l0[NP], l1[NP];
#pragma unroll
    for (int s = 0; s < NP; ++s) {
      l0[s] = part_load4(ra.part, p + s * ra.slab);
      l1[s] = part_load4(ra.part, p + s * ra.slab + 4);
    }
#pragma unroll
    for (int s = 0; s < NP; ++s) {     // slab order as splitk_reduce: bit-identical sums
      a0 += l0[s];
      a1 += l1[s];
    }
  } else {
    for (int s = 0; s < ra.nparts; ++s) {
      a0 += part_load4(ra.part, p + s * ra.slab);
      a1 += part_load4(ra.part, p + s * ra.slab + 4);
    }
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    o[j] = f2bf(a0[j]);
    o[j + 4] = f2bf(a1[j]);
  }
  return o;
}

template <int NP>
__device__ __forceinline__ bf16 qkv_load1(const RopeArgs& ra, int b, int width, int off) {
  if constexpr (NP == 0) return ra.qkv[(size_t)b * width + off];
  const size_t p = (size_t)b * width + off;
  float a = 0.f;
  if constexpr (NP > 0) {
    float l[NP];
#pragma unroll
    for (int s = 0; s < NP; ++s) l[s] = part_load1(ra.part, p + s * ra.slab);
#pragma unroll
    for (int s = 0; s < NP; ++s) a += l[s];
  } else {
    for (int s = 0; s < ra.nparts; ++s) a += part_load1(ra.part, p + s * ra.slab);
  }
  return f2bf(a);
}

template <int D, bool FUSED>
__device__ __forceinline__ void rope_rotate(bf16x8 (&f)[D / 32], const float* cs, int g) {
  if (cs == nullptr) return;
#pragma unroll
  for (int ks = 0; ks < D / 64; ++ks) {
    const f32x4 c0 = *reinterpret_cast<const f32x4*>(cs + ks * 32 + 8 * g);
    const f32x4 c1 = *reinterpret_cast<const f32x4*>(cs + ks * 32 + 8 * g + 4);
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(cs + D / 2 + ks * 32 + 8 * g);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(cs + D / 2 + ks * 32 + 8 * g + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float c = j < 4 ? c0[j] : c1[j - 4], s = j < 4 ? s0[j] : s1[j - 4];
      const float a = bf2f(f[ks][j]), b = bf2f(f[ks + D / 64][j]);
      // explicit FMAs: left to hipcc's default contraction, the fused / unfused choice here may
      // differ between kernel instantiations, and the bf16-qkv and split-K-slab forms of the fused
      // decode must rotate q / k bit-identically (a trial build rotated them 1 ulp apart at times)
      f[ks][j] = f2bf(__builtin_fmaf(a, c, -(b * s)));
      f[ks + D / 64][j] = f2bf(__builtin_fmaf(b, c, a * s));
    }
  }
}

template <int D, int WPB, bool FUSED, int PARTS = 0>
__global__ void __launch_bounds__(WPB * 64, 2) attn_decode_kernel(   // 2nd arg: min waves per SIMD
    bf16* __restrict__ out, const bf16* __restrict__ q, bf16* __restrict__ k_cache,
    bf16* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    const int32_t* __restrict__ seq_lens, float* __restrict__ part_o, float* __restrict__ part_ml,
    int hq, int hkv, int max_blocks, int split_len, float scale_log2, RopeArgs ra) {
  const int split = blockIdx.x, b = blockIdx.z;
  const int lane = threadIdx.x & 63;
  const int kvh = blockIdx.y * WPB + (threadIdx.x >> 6);
  const int nsplit = gridDim.x;
  const int G = hq / hkv;
  const int r = lane & 15, g = lane >> 4;
  // the prologue's dependency roots go out first, back to back (vmcnt retires in issue order):
  // this sequence's position (its cos / sin row), its context length and this split's first 64
  // block ids -- not guarded by the context, so they need not wait for it -- and one round trip
  // later every address the prologue loads from is known
  const int pos_b = FUSED ? ra.positions[b] : 0;
  const int ctx = seq_lens[b];
  const int kbeg = split * split_len;
  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  const int blk_first = lane < min(64, max_blocks - kbeg / kBS) ? bt[kbeg / kBS + lane] : 0;
  // FUSED: the new key (ctx - 1) is not in the cache yet: its chunk is loaded as usual and the
  // key's K row / V^T column are replaced in registers by the rotated k and v (the split that
  // owns it also appends them to the cache, after its last KV load)
  const bool owns_new = FUSED && ctx > 0 && (ctx - 1) / split_len == split;
  const int kend = min(kbeg + split_len, ctx);     // exclusive
  const int c0 = kbeg / kBS, c1 = kend > kbeg ? (kend + kBS - 1) / kBS : c0;

  // Q^T fragments: column r = head kvh*G + r (zero beyond G)
  bf16x8 qf[D / 32];
  const bool col_ok = r < G;
  bf16x8 kn[D / 32];
  bf16 vn[D / 16];
  if (FUSED) {
    const int width = (hq + 2 * hkv) * D;
    const int qo = (kvh * G + (col_ok ? r : 0)) * D, ko = (hq + kvh) * D, vo = (hq + hkv + kvh) * D;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
      qf[ks] = qkv_load8<PARTS>(ra, b, width, qo + ks * 32 + 8 * g);
      kn[ks] = qkv_load8<PARTS>(ra, b, width, ko + ks * 32 + 8 * g);
    }
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) vn[dt] = qkv_load1<PARTS>(ra, b, width, vo + dt * 16 + r);
  } else {
    const bf16* qrow = q + ((size_t)b * hq + kvh * G + (col_ok ? r : 0)) * D;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g);
      if (!col_ok) v = bf16x8{};
      qf[ks] = v;
    }
  }
  // FUSED: rotate q/k and append k/v AFTER the first KV chunk's loads are issued, so the
  // cos / sin -> rotate dependency overlaps the KV stream instead of preceding it
  bool rope_done = !FUSED;
  auto finish_rope = [&]() {
    if (!FUSED || rope_done) return;
    rope_done = true;
    const float* cs = ra.cos_sin ? ra.cos_sin + (size_t)pos_b * D : nullptr;   // pos_b: loaded first
    rope_rotate<D, FUSED>(qf, cs, g);
    rope_rotate<D, FUSED>(kn, cs, g);
    if (!col_ok) {
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) qf[ks] = bf16x8{};
    }
  };
  // FUSED: put the new key into the registers of its chunk (lane masks inside that chunk only)
  const int cnew = FUSED ? (ctx - 1) / kBS : -1;
  const int noff = FUSED ? (ctx - 1) % kBS : 0;
  auto patch = [&](KVChunk<D>& c, int chunk, size_t cbase) {
    if (!FUSED) return;
    // wave-uniform (ctx and the chunk index live in SGPRs): every other chunk skips the ~140 lane
    // selects below on a scalar branch instead of running them as no-ops
    if (!(ctx > 0 && chunk == cnew)) return;
    // (two static selects: a runtime choice between ka and kb made hipcc index them through scratch)
    const int prow = krow32(noff);                    // physical K row of the new key
    const bool krow = r == (prow & 15);
    const bool ka_row = krow && prow < 16, kb_row = krow && prow >= 16;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
      c.ka[ks] = ka_row ? kn[ks] : c.ka[ks];
      c.kb[ks] = kb_row ? kn[ks] : c.kb[ks];
    }
    // V^T fragment of lane group g: keys 8g..8g+7 -> elements 0..7
    const int e = noff & 7;
    const bool vcol = g == (noff >> 3);
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
      for (int i = 0; i < 8; ++i) c.v[dt][i] = (vcol && i == e) ? vn[dt] : c.v[dt][i];
    if constexpr (kVFullLines) {
      // append v as WHOLE lines: the 16 lanes of the new key's group hold the group's complete
      // [D][8] V^T tile (2 KiB, 16 full 128-B lines) with the new key patched in -- no partially
      // written lines to read-modify-write.  This is the sequence's last chunk: no KV load follows
      // whose vmcnt wait would include these stores.
      if (vcol && owns_new) {
#pragma unroll
        for (int dt = 0; dt < D / 16; ++dt)
          *reinterpret_cast<bf16x8*>(v_cache + cbase + g * 8 * D + (dt * 16 + r) * 8) = c.v[dt];
      }
    }
  };
  WaveState<D> st;
  init_state(st);
  const int kmax = kend - 1;
  const size_t kv_head_stride = (size_t)kBS * D;
  const size_t head_off = (size_t)kvh * kv_head_stride;
  const size_t blk_stride = (size_t)hkv * kv_head_stride;
  for (int cb = c0; cb < c1; cb += 64) {            // 64 chunks (2048 keys) of block ids per pass
    const int n = min(64, c1 - cb);
    const int my_blk = cb == c0 ? blk_first : (lane < n ? bt[cb + lane] : 0);
    KVChunk<D> cur, nxt;
    {
      const size_t base = (size_t)__builtin_amdgcn_readlane(my_blk, 0) * blk_stride + head_off;
      load_chunk<D, true>(cur, k_cache + base, v_cache + base, lane);
    }
    finish_rope();
    int j = 0;
    for (; j + 2 <= n; j += 2) {                    // ping-pong: cur <-> nxt
      {
        const size_t base = (size_t)__builtin_amdgcn_readlane(my_blk, j + 1) * blk_stride + head_off;
        load_chunk<D, true>(nxt, k_cache + base, v_cache + base, lane);
      }
      patch(cur, cb + j, (size_t)__builtin_amdgcn_readlane(my_blk, j) * blk_stride + head_off);
      compute_chunk<D>(st, qf, cur, (cb + j) * kBS, kmax, scale_log2, lane);
      if (j + 2 < n) {
        const size_t base = (size_t)__builtin_amdgcn_readlane(my_blk, j + 2) * blk_stride + head_off;
        load_chunk<D, true>(cur, k_cache + base, v_cache + base, lane);
      }
      patch(nxt, cb + j + 1, (size_t)__builtin_amdgcn_readlane(my_blk, j + 1) * blk_stride + head_off);
      compute_chunk<D>(st, qf, nxt, (cb + j + 1) * kBS, kmax, scale_log2, lane);
    }
    if (j < n) {
      patch(cur, cb + j, (size_t)__builtin_amdgcn_readlane(my_blk, j) * blk_stride + head_off);
      compute_chunk<D>(st, qf, cur, (cb + j) * kBS, kmax, scale_log2, lane);
    }
  }
  finish_rope();   // no cache chunk in this split
  if (owns_new) {
    // append k (row krow32(off)) and v (its [4][D][8] V^T slots) to the paged cache only now, after the
    // last KV load: stores count in vmcnt in issue order, so stores issued before the KV stream
    // made every later chunk wait for their (scattered 2-byte V^T) write acknowledgements
    // (cold microbench, B=256 ctx 192: 47.8 us fused vs 38.8 us attention alone)
    const int slot = ra.slots[b];
    const int blk = slot / kBS, off = slot % kBS;
    const size_t base = ((size_t)blk * hkv + kvh) * kBS * D;
    if (r == 0) {
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks)
        *reinterpret_cast<bf16x8*>(k_cache + base + (size_t)krow32(off) * D + ks * 32 + 8 * g) = kn[ks];
    }
    if (!kVFullLines && g == 0) {
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) v_cache[base + vofs(off, dt * 16 + r, D, kBS)] = vn[dt];
    }
  }
  float lt = st.lsum;
  lt = rows_sum(lt);
  if (!col_ok) return;                              // after the last MFMA: divergence is safe
  const int h = kvh * G + r;
  if (nsplit == 1) {
    // a true division, exactly as the split-reduce computes num / den (bit-identical results
    // whether a sequence's keys land in one split or in one non-empty split of several)
    bf16* orow = out + ((size_t)b * hq + h) * D;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = f2bf(lt > 0.f ? st.acc[dt][i] / lt : 0.f);
      *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = o;
    }
  } else {
    const size_t pi = ((size_t)b * hq + h) * nsplit + split;
    float* po = part_o + pi * D;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) *reinterpret_cast<f32x4*>(po + dt * 16 + 4 * g) = st.acc[dt];
    if (g == 0) { part_ml[pi * 2] = st.m; part_ml[pi * 2 + 1] = lt; }
  }
}

template <int D>
__global__ void __launch_bounds__(D) attn_split_reduce_kernel(bf16* __restrict__ out,
                                                              const float* __restrict__ part_o,
                                                              const float* __restrict__ part_ml,
                                                              int nsplit) {
  const int bh = blockIdx.x, d = threadIdx.x;
  const float* ml = part_ml + (size_t)bh * nsplit * 2;
  float M = -INFINITY;
  for (int s = 0; s < nsplit; ++s) M = fmaxf(M, ml[2 * s]);
  float num = 0.f, den = 0.f;
  if (M != -INFINITY) {
    for (int s = 0; s < nsplit; ++s) {
      const float f = exp2f(ml[2 * s] - M);
      num += part_o[((size_t)bh * nsplit + s) * D + d] * f;
      den += ml[2 * s + 1] * f;
    }
  }
  out[(size_t)bh * D + d] = f2bf(den > 0.f ? num / den : 0.f);
}

// ---------------------------------------------------------------------------
// Prefill (causal, varlen, context already in the paged cache): grid (q_tiles, Hkv, B); each wave
// owns 16/G query rows x G heads per column tile, the rows of sequence b being its LAST q_len tokens
// of ctx (chunked prefill).  Two kernels remain: the LDS-shared v4 below (default) and v3 here, its
// fallback beyond the 32k tokens of block ids v4 stages.  The first design (v1: one tile per wave,
// load -> compute per chunk, 563 us per 8B layer for 256 x 128-token prompts), v2 at one tile per
// wave and v4 at four tiles per wave (one wave per SIMD, slower) were measured and removed.
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// Prefill v3: each wave owns NT column tiles (NT x 16/G query rows x G heads) and walks the
// KV chunks with the decode kernel's depth-2 pipeline (chunk c+1's K/V loads in flight while
// chunk c's MFMAs run), so every loaded chunk serves NT tiles and its load latency is hidden.
// ---------------------------------------------------------------------------
template <int D, int G, int NT>
__global__ void __launch_bounds__(256, NT == 1 ? 2 : 1) attn_prefill2_kernel(
    bf16* __restrict__ out, const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    const int32_t* __restrict__ cu_seqlens_q, const int32_t* __restrict__ seq_lens, int hq, int hkv,
    int max_blocks, float scale_log2) {
  constexpr int R = 16 / G;                       // query rows per column tile
  const int kvh = blockIdx.y, b = blockIdx.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int qs = cu_seqlens_q[b], ql = cu_seqlens_q[b + 1] - qs;
  const int row0 = (blockIdx.x * kWaves + w) * (R * NT);
  if (row0 >= ql) return;                         // wave-uniform
  const int ctx = seq_lens[b];
  const int qpos0 = ctx - ql;                     // position of row 0
  bf16x8 qf[NT][D / 32];
  int kmax_col[NT];
  WaveState<D> st[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int crow = row0 + t * R + r / G, ch = r % G;
    const bool ok = crow < ql;
    kmax_col[t] = ok ? qpos0 + crow : -1;
    const bf16* qrow = q + ((size_t)(qs + (ok ? crow : 0)) * hq + kvh * G + ch) * D;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
      bf16x8 v = *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g);
      if (!ok) v = bf16x8{};
      qf[t][ks] = v;
    }
    init_state(st[t]);
  }
  const int wave_kmax = qpos0 + min(row0 + R * NT, ql) - 1;
  const int nch = wave_kmax / kBS + 1;            // chunks this wave reads
  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  const size_t kv_head_stride = (size_t)kBS * D;
  const size_t head_off = (size_t)kvh * kv_head_stride;
  const size_t blk_stride = (size_t)hkv * kv_head_stride;
  auto compute = [&](const KVChunk<D>& c, int chunk) {
#pragma unroll
    for (int t = 0; t < NT; ++t) compute_chunk<D>(st[t], qf[t], c, chunk * kBS, kmax_col[t], scale_log2, lane);
  };
  for (int cb = 0; cb < nch; cb += 64) {          // 64 chunks of block ids per pass
    const int n = min(64, nch - cb);
    const int my_blk = lane < n ? bt[cb + lane] : 0;
    KVChunk<D> cur, nxt;
    {
      const size_t base = (size_t)__builtin_amdgcn_readlane(my_blk, 0) * blk_stride + head_off;
      load_chunk<D>(cur, k_cache + base, v_cache + base, lane);
    }
    int j = 0;
    for (; j + 2 <= n; j += 2) {
      {
        const size_t base = (size_t)__builtin_amdgcn_readlane(my_blk, j + 1) * blk_stride + head_off;
        load_chunk<D>(nxt, k_cache + base, v_cache + base, lane);
      }
      compute(cur, cb + j);
      if (j + 2 < n) {
        const size_t base = (size_t)__builtin_amdgcn_readlane(my_blk, j + 2) * blk_stride + head_off;
        load_chunk<D>(cur, k_cache + base, v_cache + base, lane);
      }
      compute(nxt, cb + j + 1);
    }
    if (j < n) compute(cur, cb + j);
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float lt = st[t].lsum;
    lt = rows_sum(lt);
    const int crow = row0 + t * R + r / G, ch = r % G;
    if (crow < ql) {
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      bf16* orow = out + ((size_t)(qs + crow) * hq + kvh * G + ch) * D;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        bf16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = f2bf(st[t].acc[dt][i] * inv);
        *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = o;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Prefill v4 (flash-style, LDS-shared K/V): a workgroup owns kWaves x NT column tiles
// (kWaves * NT * 16/G query rows x G heads) of one (sequence, kv head) and streams the
// sequence's K/V chunks ONCE per workgroup through a 3-deep LDS ring filled by LDS-DMA
// (global_load_lds, 16 B per lane), instead of once per wave as v2 does (a 128-token prompt:
// 4x fewer K/V reads at NT = 2, 8x at NT = 4).  Per chunk: counted vmcnt for the chunk's own
// DMA pieces -> raw s_barrier -> every wave reads the chunk's fragments from LDS into the
// decode kernel's register layout -> refill the buffer all waves finished two chunks ago ->
// MFMAs (compute_chunk, shared with decode).  K is stored with a 16-B-slot XOR swizzle
// (slot ^ (row & 15), applied on the DMA source address, guide rule 21) so the K fragment
// reads are bank-conflict-free; the V^T image is already conflict-free.  Block ids are
// staged into the same LDS array first (one __shared__ object: guide trap 4a).
// ---------------------------------------------------------------------------
constexpr int kPfMaxChunks = 1024;   // 32k context per sequence

template <int D, int G, int NT, int WV = kWaves>
__global__ void __launch_bounds__(WV * 64, NT >= 4 || WV > 4 ? 1 : 2) attn_prefill_lds_kernel(
    bf16* __restrict__ out, const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    const int32_t* __restrict__ cu_seqlens_q, const int32_t* __restrict__ seq_lens, int hq, int hkv,
    int max_blocks, float scale_log2, const int32_t* __restrict__ positions, const float* __restrict__ cos_sin,
    int q_stride) {
  // q_stride: elements per token row of q ([T, hq, D]: hq * D; the raw qkv projection:
  // (hq + 2 hkv) * D).  cos_sin != null: q is the UNROTATED projection -- each lane's fragments
  // hold both rotate-half partners (dims 32 ks + 8 g + j and + D / 2), so RoPE is applied in
  // registers right after the load, as in the fused decode kernel, and the rotated q never
  // round-trips through HBM (rope_cache_kernel then appends K / V only)
  constexpr int R = 16 / G;                       // query rows per column tile
  constexpr int CH = 2 * kBS * D;                 // bf16 elements per staged chunk (K block + V^T block)
  constexpr int NB = 3;                           // ring depth
  constexpr int GL = D / 8 / WV;                  // LDS-DMA wave-instructions per wave per chunk
  static_assert(GL >= 1 && GL * WV * 512 == CH, "chunk pieces");
  constexpr int SLOTS = 2 * D / 16;               // 16-B slots per K row
  constexpr int ROWS_PER_I = 1024 / (2 * D);      // K rows per 1 KiB wave-instruction
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * CH + 2 * kPfMaxChunks];
  int* ids = reinterpret_cast<int*>(smem + NB * CH);

  // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs in dispatch order, so the
  // gridDim.x row tiles of one (sequence, kv head) -- which stream the same K / V chunks -- would
  // land on gridDim.x different XCDs (each with its own L2).  Renumber so that they share one.
  int qt = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  {
    const int nx = gridDim.x, ng = gridDim.y * gridDim.z;
    const int lin = blockIdx.x + nx * (blockIdx.y + gridDim.y * blockIdx.z);
    if (ng % 8 == 0) {
      const int xcd = lin & 7, slot = lin >> 3;            // slot-th workgroup of this XCD
      const int grp = (slot / nx) * 8 + xcd;
      qt = slot % nx;
      kvh = grp % gridDim.y;
      b = grp / gridDim.y;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const int qs = cu_seqlens_q[b], ql = cu_seqlens_q[b + 1] - qs;
  const int wg_row0 = qt * WV * R * NT;
  if (wg_row0 >= ql) return;                      // workgroup-uniform
  const int row0 = wg_row0 + w * R * NT;
  const bool active = row0 < ql;                  // wave-uniform; inactive waves still stage
  const int ctx = seq_lens[b];
  const int qpos0 = ctx - ql;
  bf16x8 qf[NT][D / 32];
  int kmax_col[NT];
  WaveState<D> st[NT];
  // q through a wave-private LDS image, the mirror of the output path below: loaded as whole
  // 16-byte pieces of columns (G heads of a row contiguous: whole lines per instruction) where the
  // fragment layout reads 64 bytes of each of 16 rows; the ring is not in use before the first
  // stage() (behind the __syncthreads below)
  constexpr int QLD = D + 8;
  constexpr bool QIMG = WV * NT * 16 * QLD <= NB * CH;
  if constexpr (QIMG) {
    bf16* img = smem + w * (NT * 16 * QLD);
    constexpr int PPC = D / 8, CPI = 64 / PPC;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int j = 0; j < 16 / CPI; ++j) {
        const int col = j * CPI + lane / PPC, piece = lane % PPC;
        const int crow = row0 + t * R + col / G, ch = col % G;
        const int tok = qs + (crow < ql ? crow : 0);
        *reinterpret_cast<bf16x8*>(img + (t * 16 + col) * QLD + piece * 8) =
            *reinterpret_cast<const bf16x8*>(q + (size_t)tok * q_stride + (size_t)(kvh * G + ch) * D + piece * 8);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int crow = row0 + t * R + r / G, ch = r % G;
    const bool ok = crow < ql;
    kmax_col[t] = ok ? qpos0 + crow : -1;
    const int tok = qs + (ok ? crow : 0);
    const bf16* qrow = q + (size_t)tok * q_stride + (size_t)(kvh * G + ch) * D;
    const bf16* irow = smem + w * (NT * 16 * QLD) + (t * 16 + r) * QLD;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
      bf16x8 v = QIMG ? *reinterpret_cast<const bf16x8*>(irow + ks * 32 + 8 * g)
                      : *reinterpret_cast<const bf16x8*>(qrow + ks * 32 + 8 * g);
      if (!ok) v = bf16x8{};
      qf[t][ks] = v;
    }
    if (cos_sin != nullptr) rope_rotate<D, true>(qf[t], cos_sin + (size_t)positions[tok] * D, g);
    init_state(st[t]);
  }
  const int wg_kmax = qpos0 + min(wg_row0 + WV * R * NT, ql) - 1;
  const int nch = wg_kmax / kBS + 1;
  const int wave_kmax = active ? qpos0 + min(row0 + R * NT, ql) - 1 : -1;
  // the smallest admissible key bound over the wave's columns (wave-uniform): -1 when any of its
  // rows is past the sequence (those columns take the masked path to stay exactly zero)
  const int wave_kmin = row0 + R * NT <= ql ? qpos0 + row0 : -1;
  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  for (int i = threadIdx.x; i < nch; i += WV * 64) ids[i] = bt[i];
  // retire the q and block-id loads before the first LDS-DMA: their uses inside the loop
  // would otherwise make hipcc wait vmcnt(0) there, draining the ring every chunk
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) asm volatile("" ::"v"(qf[t][ks]));
  __syncthreads();

  const size_t kv_head_stride = (size_t)kBS * D;
  const size_t head_off = (size_t)kvh * kv_head_stride;
  const size_t blk_stride = (size_t)hkv * kv_head_stride;
  // wave w issues 1 KiB pieces w*GL .. w*GL+GL-1 of the chunk (pieces 0..D/16-1: K, the rest: V^T)
  auto stage = [&](int c, int buf) {
    const size_t base = (size_t)ids[c] * blk_stride + head_off;
    bf16* dst = smem + buf * CH;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      const int i = w * GL + j;                   // 1 KiB piece of the 2 * 32 * D * 2 B chunk
      const bf16* src;
      if (i < D / 16) {                           // K block, swizzled slots
        const int rr = i * ROWS_PER_I + lane / SLOTS, cs = lane % SLOTS;
        src = k_cache + base + (size_t)rr * D + (cs ^ (rr & (SLOTS - 1))) * 8;
      } else {                                    // V^T block, linear
        src = v_cache + base + (size_t)(i - D / 16) * 512 + lane * 8;
      }
      __builtin_amdgcn_global_load_lds((glb_vptr_a)src, (lds_vptr_a)(dst + i * 512), 16, 0, 0);
    }
  };
  auto read = [&](KVChunk<D>& c, int buf) {
    const bf16* kb = smem + buf * CH;
    const bf16* vb = kb + kBS * D;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) {
      const int cs = ks * 4 + g;
      c.ka[ks] = *reinterpret_cast<const bf16x8*>(kb + r * D + (cs ^ (r & (SLOTS - 1))) * 8);
      c.kb[ks] = *reinterpret_cast<const bf16x8*>(kb + (16 + r) * D + (cs ^ ((16 + r) & (SLOTS - 1))) * 8);
    }
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) c.v[dt] = *reinterpret_cast<const bf16x8*>(vb + g * 8 * D + (dt * 16 + r) * 8);
  };

  stage(0, 0);
  if (nch > 1) stage(1, 1);
  int buf = 0;
  for (int c = 0; c < nch; ++c) {
    if (c + 1 < nch) {
      if constexpr (GL == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else if constexpr (GL == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    KVChunk<D> kc;
    read(kc, buf);
    // buffer (c + 2) % NB was read in iteration c - 1, which every wave finished before the
    // barrier above (its fragments were consumed by MFMAs)
    if (c + 2 < nch) stage(c + 2, buf == 0 ? NB - 1 : buf - 1);
    if (c * kBS + kBS - 1 <= wave_kmin) {         // below every column's diagonal: no mask
#pragma unroll
      for (int t = 0; t < NT; ++t) compute_chunk<D, false>(st[t], qf[t], kc, c * kBS, kmax_col[t], scale_log2, lane);
    } else if (c * kBS <= wave_kmax) {
#pragma unroll
      for (int t = 0; t < NT; ++t) compute_chunk<D>(st[t], qf[t], kc, c * kBS, kmax_col[t], scale_log2, lane);
    }
    buf = buf == NB - 1 ? 0 : buf + 1;
  }
  // Output through a wave-private LDS image (the K / V ring is free once every wave is past its
  // last chunk): a lane holds 4 dims of one column per fragment, so direct stores write 32 bytes
  // into each of 16 rows per instruction; read back as whole 16-byte pieces of a column, a store
  // instruction covers 512 / D complete columns -- with G heads of a row contiguous, whole lines.
  constexpr int OLD = D + 8;                        // padded image row (bf16): 16-B aligned, 2-way banks
  if constexpr (WV * NT * 16 * OLD > NB * CH) {     // (4 tiles per wave at D = 64: direct stores)
    if (!active) return;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      float lt = st[t].lsum;
      lt = rows_sum(lt);
      const int crow = row0 + t * R + r / G, ch = r % G;
      if (crow < ql) {
        const float inv = lt > 0.f ? 1.f / lt : 0.f;
        bf16* orow = out + ((size_t)(qs + crow) * hq + kvh * G + ch) * D;
#pragma unroll
        for (int dt = 0; dt < D / 16; ++dt) {
          bf16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = f2bf(st[t].acc[dt][i] * inv);
          *reinterpret_cast<bf16x4*>(orow + dt * 16 + 4 * g) = o;
        }
      }
    }
    return;
  }
  __syncthreads();
  if (!active) return;
  bf16* img = smem + w * (NT * 16 * OLD);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    float lt = st[t].lsum;
    lt = rows_sum(lt);
    const float inv = lt > 0.f ? 1.f / lt : 0.f;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = f2bf(st[t].acc[dt][i] * inv);
      *reinterpret_cast<bf16x4*>(img + (t * 16 + r) * OLD + dt * 16 + 4 * g) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0): the wave's own image writes landed
  __builtin_amdgcn_wave_barrier();
  constexpr int PPC = D / 8;                        // 16-byte pieces per column
  constexpr int CPI = 64 / PPC;                     // columns per store instruction
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int j = 0; j < 16 / CPI; ++j) {
      const int col = j * CPI + lane / PPC, piece = lane % PPC;
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + (t * 16 + col) * OLD + piece * 8);
      const int crow = row0 + t * R + col / G, ch = col % G;
      if (crow < ql)
        *reinterpret_cast<bf16x8*>(out + ((size_t)(qs + crow) * hq + kvh * G + ch) * D + piece * 8) = v;
    }
  }
}

// ---------------------------------------------------------------------------
// Prefill v6: v4's LDS-shared K / V stream on the 32x32x16 MFMA (v_mfma_f32_32x32x16_bf16).
// S^T = K Q^T per 64-key tile (two 32-key blocks): a lane holds 32 scores of ONE column (query row
// x head) -- 16 per block, rows 8 j + 4 hi + i of the 32x32 result -- so the column max is in-lane
// plus one v_permlane32_swap, and the per-column softmax work (max, alpha, denominator update,
// accumulator rescale) is paid once per 64 keys x 32 columns where the 16x16 form pays it per
// 32 keys x 16 columns: about half the VALU per score, and long prefill attention is VALU-bound
// (profiles/round5_prefill_attn_valu.md).
// The QK^T A operand loads key pi(m) (m with bits 2 and 3 swapped) into MFMA row m.  That puts a
// lane's 16 scores of block bb, in register order r = 8 h + 0..7, on keys 16 h + 8 hi + 0..7: the
// P.V B operand of MFMA (bb, h) is the bf16 conversion of 8 consecutive score registers (P never
// leaves the lane), and its V^T A operand is one 16-byte read of key group 2 h + hi of the cache's
// [4][D][8] V^T block.  Workgroup: 8 waves x 32 columns (32 / G query rows x G heads each) of one
// (sequence, kv head); K / V tiles stream through a 3-deep LDS ring by LDS-DMA with v4's XOR-swizzled
// K rows, conflict-free for this read pattern as well (the 16 lanes of a ds_read_b128 group hit 16
// distinct row & 15 values).
// ---------------------------------------------------------------------------
constexpr int kW32Waves = 8;

// physical K row (common.h krow32 layout) of the key pi(m) the QK^T A operand puts at MFMA row m
__device__ __forceinline__ int w32_krow(int m) {
  return (((m >> 3) & 1) << 4) | ((m >> 4) << 3) | (((m >> 2) & 1) << 2) | (m & 3);
}

// max / sum with the lane 32 apart (the other half of a 32x32 accumulator column)
__device__ __forceinline__ float half_max(float v) {
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float half_sum(float v) {
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

template <int G, bool PIPE>
__global__ void __launch_bounds__(kW32Waves * 64, 1) attn_prefill_w32_kernel(
    bf16* __restrict__ out, const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    const int32_t* __restrict__ cu_seqlens_q, const int32_t* __restrict__ seq_lens, int hq, int hkv,
    int max_blocks, float scale_log2, const int32_t* __restrict__ positions, const float* __restrict__ cos_sin,
    int q_stride) {
  constexpr int D = 128;
  constexpr int WV = kW32Waves;
  constexpr int R = 32 / G;                       // query rows per wave
  constexpr int TK = 2 * kBS;                     // keys per tile
  constexpr int BLK = kBS * D;                    // bf16 elements of one K block (= one V^T block)
  constexpr int TILE = 4 * BLK;                   // K0 K1 V0 V1: 32 KiB
  constexpr int NB = PIPE ? 4 : 3;                // ring depth
  constexpr int GL = TILE / 512 / WV;             // 1 KiB LDS-DMA pieces per wave per tile
  static_assert(GL == 4 && 32 % G == 0, "tile pieces / column tiling");
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * TILE + 2 * kPfMaxChunks];
  int* ids = reinterpret_cast<int*>(smem + NB * TILE);

  // XCD-aware order (as v4): the row tiles of one (sequence, kv head) share an XCD's L2; and the
  // last row tiles -- the most keys under the causal mask -- are dispatched first, so the long
  // workgroups do not form the launch's tail
  int qt = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  {
    const int nx = gridDim.x, ng = gridDim.y * gridDim.z;
    const int lin = blockIdx.x + nx * (blockIdx.y + gridDim.y * blockIdx.z);
    if (ng % 8 == 0) {
      const int xcd = lin & 7, slot = lin >> 3;
      const int grp = (slot / nx) * 8 + xcd;
      qt = slot % nx;
      kvh = grp % gridDim.y;
      b = grp / gridDim.y;
    }
    qt = nx - 1 - qt;
  }
  // the wave index through readfirstlane: hipcc then knows it (and every bound derived from it) is
  // wave-uniform and branches on it with scalar branches instead of EXEC masks
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = lane & 31, hi = lane >> 5;
  const int qs = cu_seqlens_q[b], ql = cu_seqlens_q[b + 1] - qs;
  const int wg_row0 = qt * WV * R;
  if (wg_row0 >= ql) return;                      // workgroup-uniform
  const int row0 = wg_row0 + w * R;
  const bool active = row0 < ql;                  // wave-uniform; inactive waves still stage
  const int ctx = seq_lens[b];
  const int qpos0 = ctx - ql;
  // this lane's column: query row row0 + m / G, head kvh * G + m % G
  const int crow = row0 + m / G, ch = m % G;
  const bool ok = crow < ql;
  const int kmax_col = ok ? qpos0 + crow : -1;
  const int tok = qs + (ok ? crow : 0);
  // Q^T fragments (B operand): column m, dims 16 ks + 8 hi + 0..7; RoPE partners (d, d + 64) are
  // fragments ks and ks + 4 of the same lane
  bf16x8 qf[D / 16];
  {
    const bf16* qrow = q + (size_t)tok * q_stride + (size_t)(kvh * G + ch) * D + 8 * hi;
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + 16 * ks);
    if (cos_sin != nullptr) {
      const float* cs = cos_sin + (size_t)positions[tok] * D + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) {
        const f32x4 c0 = *reinterpret_cast<const f32x4*>(cs + 16 * ks);
        const f32x4 c1 = *reinterpret_cast<const f32x4*>(cs + 16 * ks + 4);
        const f32x4 s0 = *reinterpret_cast<const f32x4*>(cs + D / 2 + 16 * ks);
        const f32x4 s1 = *reinterpret_cast<const f32x4*>(cs + D / 2 + 16 * ks + 4);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float c = j < 4 ? c0[j] : c1[j - 4], s = j < 4 ? s0[j] : s1[j - 4];
          const float a = bf2f(qf[ks][j]), bq = bf2f(qf[ks + D / 32][j]);
          qf[ks][j] = f2bf(__builtin_fmaf(a, c, -(bq * s)));   // as rope_rotate: explicit FMAs
          qf[ks + D / 32][j] = f2bf(__builtin_fmaf(bq, c, a * s));
        }
      }
    }
    if (!ok) {
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) qf[ks] = bf16x8{};
    }
  }
  const int wg_kmax = qpos0 + min(wg_row0 + WV * R, ql) - 1;
  const int nch = wg_kmax / kBS + 1;              // 32-key blocks the workgroup reads
  const int ntile = (nch + 1) / 2;
  const int wave_kmax = active ? qpos0 + min(row0 + R, ql) - 1 : -1;
  const int wave_kmin = row0 + R <= ql ? qpos0 + row0 : -1;   // -1: a column past the sequence
  const int32_t* bt = block_tables + (size_t)b * max_blocks;
  for (int i = threadIdx.x; i < nch; i += WV * 64) ids[i] = bt[i];
  // retire the q loads before the first LDS-DMA (a use inside the loop would wait vmcnt(0) there)
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) asm volatile("" ::"v"(qf[ks]));
  __syncthreads();

  const size_t head_off = (size_t)kvh * BLK;
  const size_t blk_stride = (size_t)hkv * BLK;
  // wave w stages 1 KiB pieces 4 w .. 4 w + 3 of tile t: pieces 0-7 K block 0, 8-15 K block 1,
  // 16-23 V^T block 0, 24-31 V^T block 1 (a block past the sequence re-reads the last one: its keys
  // are masked for every column)
  // (a wave's four pieces are one part: one block id per wave, read once and made scalar)
  auto stage = [&](int t, int buf) {
    bf16* dst = smem + buf * TILE;
    static_assert(GL * 2 == 8, "one part per wave");
    const int c = min(2 * t + ((w >> 1) & 1), nch - 1);
    const size_t base = (size_t)__builtin_amdgcn_readfirstlane(ids[c]) * blk_stride + head_off;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      const int i = w * GL + j, part = i >> 3;
      const bf16* src;
      if (part < 2) {
        const int rr = (i & 7) * 4 + lane / 16, cs = lane % 16;
        src = k_cache + base + (size_t)rr * D + (cs ^ (rr & 15)) * 8;
      } else {
        src = v_cache + base + (size_t)(i & 7) * 512 + lane * 8;
      }
      __builtin_amdgcn_global_load_lds((glb_vptr_a)src, (lds_vptr_a)(dst + i * 512), 16, 0, 0);
    }
  };
  const int krow = w32_krow(m), kswz = krow & 15;
  f32x16 acc[D / 32];                             // O^T: dims 32 dt + 8 (r / 4) + 4 hi + r % 4, column m
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) acc[dt] = f32x16{};
  float mrun = -INFINITY, lsum = 0.f;
  const f32x2 sc2 = {scale_log2, scale_log2};

  // S^T of tile tb (two blocks): 16 MFMAs reading K fragments from the ring
  auto qk = [&](const bf16* tb, f32x16& s0, f32x16& s1) {
    s0 = f32x16{};
    s1 = f32x16{};
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) {
      const int slot = ((2 * ks + hi) ^ kswz) * 8;
      const bf16x8 ka = *reinterpret_cast<const bf16x8*>(tb + krow * D + slot);
      const bf16x8 kb = *reinterpret_cast<const bf16x8*>(tb + BLK + krow * D + slot);
      s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], s0, 0, 0, 0);
      s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb, qf[ks], s1, 0, 0, 0);
    }
  };
  // causal mask: register r of block bb holds key k0 + 32 bb + 16 (r >> 3) + 8 hi + (r & 7).  Behind a
  // wave-uniform branch in ONE instantiation: two (masked / unmasked) copies of the tile made hipcc
  // keep the accumulators in different registers per copy and shuffle all 64 (v_mov_b64 x 32) at merges
  auto mask = [&](f32x16& s0, f32x16& s1, int k0) {
    const int kl = kmax_col - k0 - 8 * hi;         // admissible: 16 (r >> 3) + (r & 7) (+ 32) <= kl
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = 16 * (r >> 3) + (r & 7);
      s0[r] = key <= kl ? s0[r] : -INFINITY;
      s1[r] = key + kBS <= kl ? s1[r] : -INFINITY;
    }
  };
  // online softmax of one tile's scores: the P.V B operands pb[2 bb + h], the rescale factor
  auto softmax = [&](const f32x16& s0, const f32x16& s1, bf16x8 (&pb)[4]) {
    float cm = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) cm = fmaxf(cm, fmaxf(s0[r], s1[r]));
    cm = half_max(cm) * scale_log2;
    const float mn = fmaxf(mrun, cm);
    const float mref = (mn == -INFINITY) ? 0.f : mn;
    const float alpha = __builtin_amdgcn_exp2f(mrun - mref);
    mrun = mn;
    const f32x2 mr2 = {-mref, -mref};
    f32x2 sum2 = {0.f, 0.f};
#pragma unroll
    for (int p = 0; p < 16; ++p) {                 // score pairs: block p / 8, registers 2 (p % 8) + 0, 1
      const f32x16& sv = p < 8 ? s0 : s1;
      const int r = 2 * (p & 7);
      const f32x2 x = __builtin_elementwise_fma(f32x2{sv[r], sv[r + 1]}, sc2, mr2);
      const f32x2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
      sum2 += e;
      pb[p >> 2][r & 7] = f2bf(e[0]);
      pb[p >> 2][(r & 7) + 1] = f2bf(e[1]);
    }
    lsum = lsum * alpha + (sum2[0] + sum2[1]);
    return alpha;
  };
  auto rescale = [&](float alpha) {
    if (__any(alpha != 1.f)) {                      // exactly 1 wherever no column's max moved
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) acc[dt] *= alpha;
    }
  };
  // O^T += V^T P^T for the tile in ring slot tb: 16 MFMAs reading V^T fragments from the ring
  auto pv = [&](const bf16* tb, const bf16x8 (&pb)[4]) {
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
      for (int bh = 0; bh < 4; ++bh) {
        const bf16x8 va = *reinterpret_cast<const bf16x8*>(
            tb + 2 * BLK + (bh >> 1) * BLK + ((2 * (bh & 1) + hi) * D + 32 * dt + m) * 8);
        acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pb[bh], acc[dt], 0, 0, 0);
      }
    }
  };

  stage(0, 0);
  if (ntile > 1) stage(1, 1);
  // PIPE: the previous tile's P.V MFMAs go out right behind this tile's QK^T and run while the VALU
  // does this tile's softmax (MFMA and VALU are separate pipes; without it a wave's P.V waits for
  // its own softmax, and only the other wave on the SIMD can fill the gap).  The ring is one deeper:
  // a tile's V^T is still read one iteration after its K.  An active wave runs every tile of the
  // workgroup (past its own rows' keys the scores are all masked: P = 0, alpha = 1) so that the
  // accumulators see one straight-line path per iteration -- a skip path made hipcc copy all 64 of
  // them in and out of the tile code
  bf16x8 pbp[4] = {};                             // PIPE: P of the previous tile (zeros: a no-op P.V)
  int vprev = 0;                                  // PIPE: its ring slot
  for (int t = 0; t < ntile; ++t) {
    if (t + 1 < ntile) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // slot (t + 2) % NB was last read in iteration t - 1 (PIPE: t - 2's V^T in iteration t - 1), which
    // every wave finished before the barrier
    const bf16* tb = smem + (t % NB) * TILE;
    const int k0 = t * TK;
    if constexpr (PIPE) {
      // PIPE stages behind this tile's QK^T: the block-id read and address work then run under the
      // MFMAs instead of between the barrier and the first of them
      if (!active) {
        if (t + 2 < ntile) stage(t + 2, (t + 2) % NB);
        continue;
      }
      f32x16 s0, s1;
      qk(tb, s0, s1);
      __builtin_amdgcn_sched_barrier(0);
      if (t + 2 < ntile) stage(t + 2, (t + 2) % NB);
      if (k0 + TK - 1 > wave_kmin) mask(s0, s1, k0);   // unmasked below every column's diagonal
      // the previous tile's 16 P.V MFMAs with this tile's softmax in their gaps, one slice per gap
      // (sched_barrier(0) fences each gap): gaps 0-3 the column max over registers 4 k .. 4 k + 3 of
      // both blocks, gap 4 the cross-half max and the running-max update, gaps 5-15 the 16 score pairs
      // (FMA, two exp, cvt, sum).  MFMA i: d-tile i & 3 (consecutive MFMAs on different accumulators),
      // P operand i >> 2; its V^T fragment is read one group of four ahead.
      const bf16* vt = smem + vprev * TILE;
      auto vread = [&](int i) {
        const int dt = i & 3, bh = i >> 2;
        return *reinterpret_cast<const bf16x8*>(vt + 2 * BLK + (bh >> 1) * BLK +
                                                ((2 * (bh & 1) + hi) * D + 32 * dt + m) * 8);
      };
      bf16x8 va[4], vn[4], pb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) va[j] = vread(j);
      float cmp[4], alpha = 1.f, mref = 0.f;
      f32x2 sum2 = {0.f, 0.f};
      auto pair = [&](int p) {                     // score pair p: block p / 8, registers 2 (p % 8) + 0, 1
        const f32x16& sv = p < 8 ? s0 : s1;
        const int r = 2 * (p & 7);
        const f32x2 x = __builtin_elementwise_fma(f32x2{sv[r], sv[r + 1]}, sc2, f32x2{-mref, -mref});
        const f32x2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
        sum2 += e;
        pb[p >> 2][r & 7] = f2bf(e[0]);
        pb[p >> 2][(r & 7) + 1] = f2bf(e[1]);
      };
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if ((i & 3) == 0 && i + 4 < 16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) vn[j] = vread(i + 4 + j);
        }
        acc[i & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[i & 3], pbp[i >> 2], acc[i & 3], 0, 0, 0);
        if ((i & 3) == 3 && i + 1 < 16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) va[j] = vn[j];
        }
        if (i < 4) {
          cmp[i] = fmaxf(fmaxf(fmaxf(s0[4 * i], s0[4 * i + 1]), fmaxf(s0[4 * i + 2], s0[4 * i + 3])),
                         fmaxf(fmaxf(s1[4 * i], s1[4 * i + 1]), fmaxf(s1[4 * i + 2], s1[4 * i + 3])));
        } else if (i == 4) {
          const float cm = half_max(fmaxf(fmaxf(cmp[0], cmp[1]), fmaxf(cmp[2], cmp[3]))) * scale_log2;
          const float mn = fmaxf(mrun, cm);
          mref = (mn == -INFINITY) ? 0.f : mn;
          alpha = __builtin_amdgcn_exp2f(mrun - mref);
          mrun = mn;
        } else if (i < 10) {
          pair(2 * (i - 5));
          pair(2 * (i - 5) + 1);
        } else {
          pair(i);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      // pin the probabilities and their sum here: hipcc would otherwise sink the exp / cvt / add work
      // past the rescale branch below, out of the MFMAs' shadow
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(pb[i]));
      asm volatile("" : "+v"(sum2));
      lsum = lsum * alpha + (sum2[0] + sum2[1]);
      rescale(alpha);
#pragma unroll
      for (int i = 0; i < 4; ++i) pbp[i] = pb[i];
      vprev = t % NB;
    } else if (t + 2 < ntile) {
      stage(t + 2, (t + 2) % NB);
    }
    if (!PIPE && k0 <= wave_kmax) {
      f32x16 s0, s1;
      qk(tb, s0, s1);
      if (k0 + TK - 1 > wave_kmin) mask(s0, s1, k0);
      bf16x8 pb[4];
      rescale(softmax(s0, s1, pb));
      pv(tb, pb);
    }
  }
  if (PIPE && active) pv(smem + vprev * TILE, pbp);
  const float lt = half_sum(lsum);
  // output through a wave-private LDS image (the ring is free once every wave is past its last
  // tile): whole 16-byte pieces of a column per store, G heads of a row contiguous -- whole lines
  constexpr int OLD = D + 8;
  static_assert(WV * 32 * OLD <= NB * TILE, "output image");
  __syncthreads();
  if (!active) return;
  bf16* img = smem + w * (32 * OLD);
  const float inv = lt > 0.f ? 1.f / lt : 0.f;
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[dt][4 * j + i] * inv);
      *reinterpret_cast<bf16x4*>(img + m * OLD + 32 * dt + 8 * j + 4 * hi) = o;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);               // lgkmcnt(0): the wave's own image writes landed
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int it = 0; it < 32 * (D / 8) / 64; ++it) {
    const int p = it * 64 + lane, col = p / (D / 8), piece = p % (D / 8);
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + col * OLD + piece * 8);
    const int crow2 = row0 + col / G, ch2 = col % G;
    if (crow2 < ql)
      *reinterpret_cast<bf16x8*>(out + ((size_t)(qs + crow2) * hq + kvh * G + ch2) * D + piece * 8) = v;
  }
}

// ---------------------------------------------------------------------------
// Prefill v9: v7 made persistent.  A fit of v7's times from 128- to 16k-token prompts gives ~12 us
// per 64-row workgroup on top of the streaming work (prologue, first-tile latency, output), and with
// one 8-wave workgroup per CU nothing else runs meanwhile.  Here one workgroup per CU walks row tiles
// ("items") of its XCD's (sequence, kv head) groups -- group g on XCD g % 8, as v7's order -- in a
// snake over heavy-first order (round r of the XCD's PX workgroups runs left to right, r + 1 right to
// left: a workgroup's heavy and light row tiles pair up).  The LDS ring runs on a global tile count
// across items: the next item's first two K / V tiles are staged under the current item's last two
// (their block ids straight from the table), so an item starts on landed data; its q loads and the
// previous item's output stores are the only latency left at a switch.  Output goes straight from
// the accumulators (the ring is busy): the two half-waves swap dword pairs with v_permlane32_swap so
// that every lane stores 16 contiguous bytes of its column.
// ---------------------------------------------------------------------------
template <int G>
__global__ void __launch_bounds__(kW32Waves * 64, 1) attn_prefill_w32p_kernel(
    bf16* __restrict__ out, const bf16* __restrict__ q, const bf16* __restrict__ k_cache,
    const bf16* __restrict__ v_cache, const int32_t* __restrict__ block_tables,
    const int32_t* __restrict__ cu_seqlens_q, const int32_t* __restrict__ seq_lens, int hq, int hkv,
    int max_blocks, float scale_log2, const int32_t* __restrict__ positions, const float* __restrict__ cos_sin,
    int q_stride, int nx, int ngroups) {
  constexpr int D = 128;
  constexpr int WV = kW32Waves;
  constexpr int R = 32 / G;                       // query rows per wave
  constexpr int RWG = WV * R;                     // query rows per item
  constexpr int TK = 2 * kBS;
  constexpr int BLK = kBS * D;
  constexpr int TILE = 4 * BLK;
  constexpr int NB = 4;
  constexpr int GL = TILE / 512 / WV;
  static_assert(GL == 4 && 32 % G == 0, "tile pieces / column tiling");
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * TILE + 4 * kPfMaxChunks];
  int* ids = reinterpret_cast<int*>(smem + NB * TILE);   // two block-id lists: this item's, the next's

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int m = lane & 31, hi = lane >> 5;
  const int xcd = blockIdx.x & 7, wx = blockIdx.x >> 3, PX = gridDim.x >> 3;
  const int gx = ngroups > xcd ? (ngroups - 1 - xcd) / 8 + 1 : 0;   // groups on this XCD
  const int nitems = gx * nx;

  struct Item {
    int b, kvh, qs, ql, qpos0, row0, ntile, nch;
  };
  // r-th item of this workgroup (snake over rounds); false past the end
  auto pos_of = [&](int r) { return r * PX + ((r & 1) ? PX - 1 - wx : wx); };
  auto load_item = [&](int p, Item& it) {
    const int gi = p / nx, qt = nx - 1 - p % nx;
    const int g = xcd + 8 * gi;
    it.b = g / hkv;
    it.kvh = g % hkv;
    it.qs = cu_seqlens_q[it.b];
    it.ql = cu_seqlens_q[it.b + 1] - it.qs;
    it.row0 = qt * RWG;
    const int ctx = seq_lens[it.b];
    it.qpos0 = ctx - it.ql;
    const int kmax = it.qpos0 + min(it.row0 + RWG, it.ql) - 1;
    it.nch = kmax / kBS + 1;
    it.ntile = (it.nch + 1) / 2;
    return it.row0 < it.ql;                       // rows past the sequence: an empty item
  };
  // the next non-empty item at or after round r: its round, or -1
  auto next_item = [&](int r, Item& it) {
    for (; pos_of(r) < nitems; ++r)
      if (load_item(pos_of(r), it)) return r;
    return -1;
  };

  Item cur, nxt;
  int rc = next_item(0, cur);
  if (rc < 0) return;                             // workgroup-uniform
  int rn = next_item(rc + 1, nxt);

  const size_t blk_stride = (size_t)hkv * BLK;
  // stage local tile t of item it, block ids in list il, into ring slot buf.  The ids come from
  // LDS: the next item's list is written in this item's prologue, so its first tiles can be staged
  // under this item's last ones.  (Reading them from the table for the first tiles instead made a
  // select between a global and an LDS pointer, a flat load, whose wait drains the DMA just issued.)
  auto stage = [&](const Item& it, int il, int t, int buf) {
    bf16* dst = smem + buf * TILE;
    const size_t head_off = (size_t)it.kvh * BLK;
    const int c = min(2 * t + ((w >> 1) & 1), it.nch - 1);
    const int id = __builtin_amdgcn_readfirstlane(ids[il * kPfMaxChunks + c]);
    const size_t base = (size_t)id * blk_stride + head_off;
#pragma unroll
    for (int j = 0; j < GL; ++j) {
      const int i = w * GL + j, part = i >> 3;
      const bf16* src;
      if (part < 2) {
        const int rr = (i & 7) * 4 + lane / 16, cs = lane % 16;
        src = k_cache + base + (size_t)rr * D + (cs ^ (rr & 15)) * 8;
      } else {
        src = v_cache + base + (size_t)(i & 7) * 512 + lane * 8;
      }
      __builtin_amdgcn_global_load_lds((glb_vptr_a)src, (lds_vptr_a)(dst + i * 512), 16, 0, 0);
    }
  };
  // global tile gt + d, where cur's tile 0 is global tile g0: cur's, else nxt's, else none
  int g0 = 0, staged = 0;                         // global tiles [0, staged) have been issued
  int il = 0;                                     // cur's block-id list (nxt's: il ^ 1)
  // nxt's tiles only from inside cur's tile loop: nxt's list is written in cur's prologue
  auto stage_global = [&](int gidx, bool may_next) {
    const int lt = gidx - g0;
    if (lt < cur.ntile) {
      stage(cur, il, lt, gidx % NB);
    } else if (may_next && rn >= 0 && lt - cur.ntile < nxt.ntile) {
      stage(nxt, il ^ 1, lt - cur.ntile, gidx % NB);
    } else {
      return;
    }
    staged = gidx + 1;
  };
  {
    const int32_t* bt = block_tables + (size_t)cur.b * max_blocks;
    for (int i = threadIdx.x; i < cur.nch; i += WV * 64) ids[i] = bt[i];
  }
  __syncthreads();
  stage_global(0, false);
  stage_global(1, false);

  const int krow = w32_krow(m), kswz = krow & 15;
  const f32x2 sc2 = {scale_log2, scale_log2};
  while (true) {
    // ---- item prologue: this lane's column, q (rotated), LDS block ids of tiles >= 2
    const int row0 = cur.row0 + w * R;
    const bool active = row0 < cur.ql;
    const int crow = row0 + m / G, ch = m % G;
    const bool ok = crow < cur.ql;
    const int kmax_col = ok ? cur.qpos0 + crow : -1;
    const int tok = cur.qs + (ok ? crow : 0);
    const int wave_kmin = row0 + R <= cur.ql ? cur.qpos0 + row0 : -1;
    bf16x8 qf[D / 16];
    {
      const bf16* qrow = q + (size_t)tok * q_stride + (size_t)(cur.kvh * G + ch) * D + 8 * hi;
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qrow + 16 * ks);
      if (cos_sin != nullptr) {
        const float* cs = cos_sin + (size_t)positions[tok] * D + 8 * hi;
#pragma unroll
        for (int ks = 0; ks < D / 32; ++ks) {
          const f32x4 c0 = *reinterpret_cast<const f32x4*>(cs + 16 * ks);
          const f32x4 c1 = *reinterpret_cast<const f32x4*>(cs + 16 * ks + 4);
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(cs + D / 2 + 16 * ks);
          const f32x4 s1 = *reinterpret_cast<const f32x4*>(cs + D / 2 + 16 * ks + 4);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float c = j < 4 ? c0[j] : c1[j - 4], s = j < 4 ? s0[j] : s1[j - 4];
            const float a = bf2f(qf[ks][j]), bq = bf2f(qf[ks + D / 32][j]);
            qf[ks][j] = f2bf(__builtin_fmaf(a, c, -(bq * s)));
            qf[ks + D / 32][j] = f2bf(__builtin_fmaf(bq, c, a * s));
          }
        }
      }
      if (!ok) {
#pragma unroll
        for (int ks = 0; ks < D / 16; ++ks) qf[ks] = bf16x8{};
      }
    }
    if (rn >= 0) {                                  // the next item's block ids (its list was the
      const int32_t* bt = block_tables + (size_t)nxt.b * max_blocks;   // previous item's: all read)
      int* dst = ids + (il ^ 1) * kPfMaxChunks;
      for (int i = threadIdx.x; i < nxt.nch; i += WV * 64) dst[i] = bt[i];
    }
    // everything issued so far (q, ids, this item's first tiles, the previous item's stores) lands
    // here: the tile loop's counted waits then see only its own LDS-DMA
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks) asm volatile("" ::"v"(qf[ks]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    f32x16 acc[D / 32];
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) acc[dt] = f32x16{};
    float mrun = -INFINITY, lsum = 0.f;
    bf16x8 pbp[4] = {};
    int vprev = g0 % NB;
    for (int t = 0; t < cur.ntile; ++t) {
      const int gidx = g0 + t;
      if (staged > gidx + 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      // ring slot (gidx + 2) % NB was last read in iteration gidx - 1 (its V^T), finished by every wave;
      // active waves stage it behind this tile's QK^T MFMAs
      // (gidx + 1 too when a one-tile item left it unstaged: its slot was read in iterations gidx - 3
      // and gidx - 2)
      if (!active) {
        if (staged == gidx + 1) stage_global(gidx + 1, true);
        if (staged == gidx + 2) stage_global(gidx + 2, true);
        continue;
      }
      const bf16* tb = smem + (gidx % NB) * TILE;
      const int k0 = t * TK;
      f32x16 s0 = {}, s1 = {};
#pragma unroll
      for (int ks = 0; ks < D / 16; ++ks) {
        const int slot = ((2 * ks + hi) ^ kswz) * 8;
        const bf16x8 ka = *reinterpret_cast<const bf16x8*>(tb + krow * D + slot);
        const bf16x8 kb = *reinterpret_cast<const bf16x8*>(tb + BLK + krow * D + slot);
        s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka, qf[ks], s0, 0, 0, 0);
        s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kb, qf[ks], s1, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (staged == gidx + 1) stage_global(gidx + 1, true);
      if (staged == gidx + 2) stage_global(gidx + 2, true);
      if (k0 + TK - 1 > wave_kmin) {
        const int kl = kmax_col - k0 - 8 * hi;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = 16 * (r >> 3) + (r & 7);
          s0[r] = key <= kl ? s0[r] : -INFINITY;
          s1[r] = key + kBS <= kl ? s1[r] : -INFINITY;
        }
      }
      const bf16* vt = smem + vprev * TILE;
      auto vread = [&](int i) {
        const int dt = i & 3, bh = i >> 2;
        return *reinterpret_cast<const bf16x8*>(vt + 2 * BLK + (bh >> 1) * BLK +
                                                ((2 * (bh & 1) + hi) * D + 32 * dt + m) * 8);
      };
      bf16x8 va[4], vn[4], pb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) va[j] = vread(j);
      float cmp[4], alpha = 1.f, mref = 0.f;
      f32x2 sum2 = {0.f, 0.f};
      auto pair = [&](int p) {
        const f32x16& sv = p < 8 ? s0 : s1;
        const int r = 2 * (p & 7);
        const f32x2 x = __builtin_elementwise_fma(f32x2{sv[r], sv[r + 1]}, sc2, f32x2{-mref, -mref});
        const f32x2 e = {__builtin_amdgcn_exp2f(x[0]), __builtin_amdgcn_exp2f(x[1])};
        sum2 += e;
        pb[p >> 2][r & 7] = f2bf(e[0]);
        pb[p >> 2][(r & 7) + 1] = f2bf(e[1]);
      };
#pragma unroll
      for (int i = 0; i < 16; ++i) {                // as v7: the previous tile's P.V under this softmax
        if ((i & 3) == 0 && i + 4 < 16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) vn[j] = vread(i + 4 + j);
        }
        acc[i & 3] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va[i & 3], pbp[i >> 2], acc[i & 3], 0, 0, 0);
        if ((i & 3) == 3 && i + 1 < 16) {
#pragma unroll
          for (int j = 0; j < 4; ++j) va[j] = vn[j];
        }
        if (i < 4) {
          cmp[i] = fmaxf(fmaxf(fmaxf(s0[4 * i], s0[4 * i + 1]), fmaxf(s0[4 * i + 2], s0[4 * i + 3])),
                         fmaxf(fmaxf(s1[4 * i], s1[4 * i + 1]), fmaxf(s1[4 * i + 2], s1[4 * i + 3])));
        } else if (i == 4) {
          const float cm = half_max(fmaxf(fmaxf(cmp[0], cmp[1]), fmaxf(cmp[2], cmp[3]))) * scale_log2;
          const float mn = fmaxf(mrun, cm);
          mref = (mn == -INFINITY) ? 0.f : mn;
          alpha = __builtin_amdgcn_exp2f(mrun - mref);
          mrun = mn;
        } else if (i < 10) {
          pair(2 * (i - 5));
          pair(2 * (i - 5) + 1);
        } else {
          pair(i);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(pb[i]));
      asm volatile("" : "+v"(sum2));
      lsum = lsum * alpha + (sum2[0] + sum2[1]);
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < D / 32; ++dt) acc[dt] *= alpha;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) pbp[i] = pb[i];
      vprev = gidx % NB;
    }
    if (active) {
      // the last tile's P.V
      const bf16* vt = smem + vprev * TILE;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
        for (int bh = 0; bh < 4; ++bh) {
          const bf16x8 va = *reinterpret_cast<const bf16x8*>(
              vt + 2 * BLK + (bh >> 1) * BLK + ((2 * (bh & 1) + hi) * D + 32 * dt + m) * 8);
          acc[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(va, pbp[bh], acc[dt], 0, 0, 0);
        }
      }
      // output: lane (m, hi) holds dims 32 dt + 8 j + 4 hi + 0..3 of column m; for each pair of j
      // (2p, 2p + 1) the half-waves swap one 8-byte quad (v_permlane32_swap: lanes 32-63 of the
      // first operand <-> lanes 0-31 of the second), after which lane (m, hi) holds the 8 dims
      // 32 dt + 8 (2p + hi) + 0..7: one 16-byte store
      const float lt = half_sum(lsum);
      const float inv = lt > 0.f ? 1.f / lt : 0.f;
      bf16* orow = out + ((size_t)(cur.qs + (ok ? crow : 0)) * hq + cur.kvh * G + ch) * D;
#pragma unroll
      for (int dt = 0; dt < D / 32; ++dt) {
#pragma unroll
        for (int pp = 0; pp < 2; ++pp) {
          bf16x4 u0, u1;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            u0[i] = f2bf(acc[dt][4 * (2 * pp) + i] * inv);
            u1[i] = f2bf(acc[dt][4 * (2 * pp + 1) + i] * inv);
          }
          typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
          u32x2v a = __builtin_bit_cast(u32x2v, u0), bb = __builtin_bit_cast(u32x2v, u1);
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const auto sw = __builtin_amdgcn_permlane32_swap(a[k], bb[k], false, false);
            a[k] = sw[0];
            bb[k] = sw[1];
          }
          typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
          const u32x4v o = {a[0], a[1], bb[0], bb[1]};
          if (ok) *reinterpret_cast<u32x4v*>(orow + 32 * dt + 8 * (2 * pp + hi)) = o;
        }
      }
    }
    // ---- next item: its first tiles are staged (or in flight); move the window
    if (rn < 0) break;
    g0 += cur.ntile;
    cur = nxt;
    il ^= 1;
    rc = rn;
    rn = next_item(rc + 1, nxt);
    while (staged < g0 + 2) {                       // an item shorter than two tiles left gaps
      const int before = staged;
      stage_global(staged, false);
      if (staged == before) break;
    }
  }
}

// ------------------------------------------------------------------ launchers
static void decode_launch(uintptr_t out, uintptr_t q, uintptr_t k_cache, uintptr_t v_cache, uintptr_t block_tables,
                          uintptr_t seq_lens, uintptr_t part_o, uintptr_t part_ml, int batch, int hq, int hkv, int d,
                          int block_size, int max_blocks, int num_splits, int split_len, float scale, RopeArgs ra,
                          bool fused, uintptr_t stream) {
  DLLM_HOST_CHECK(block_size == kBS, "paged attention requires block_size 32");
  DLLM_HOST_CHECK(hq % hkv == 0 && hq / hkv <= 16, "GQA group size must be <= 16");
  DLLM_HOST_CHECK(d == 64 || d == 128, "head_dim must be 64 or 128");
  DLLM_HOST_CHECK(num_splits >= 1 && split_len % kBS == 0 && split_len > 0, "split_len multiple of 32");
  DLLM_HOST_CHECK(num_splits == 1 || (part_o && part_ml), "split workspace");
  DLLM_HOST_CHECK(!fused || ((ra.qkv || ra.part) && ra.positions && ra.slots),
                  "fused decode needs qkv, positions, slots");
  DLLM_HOST_CHECK(ra.part == nullptr || (ra.nparts >= 1 && ra.slab >= (long)batch * (hq + 2 * hkv) * d),
                  "qkv partial slabs");
  if (batch == 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float sl2 = scale * 1.4426950408889634f;
  // one wave per kv head; pack up to 4 heads (independent waves) per workgroup
  const int wpb = hkv % 4 == 0 ? 4 : hkv % 2 == 0 ? 2 : 1;
  dim3 grid(num_splits, hkv / wpb, batch);
  auto go = [&](auto kern, int threads) {
    hipLaunchKernelGGL(kern, grid, dim3(threads), 0, s, (bf16*)out, (const bf16*)q, (bf16*)k_cache, (bf16*)v_cache,
                       (const int32_t*)block_tables, (const int32_t*)seq_lens, (float*)part_o, (float*)part_ml, hq,
                       hkv, max_blocks, split_len, sl2, ra);
  };
#define DLLM_DEC(DD, FF, PP)                                          \
  do {                                                                \
    if (wpb == 4) go(attn_decode_kernel<DD, 4, FF, PP>, 256);         \
    else if (wpb == 2) go(attn_decode_kernel<DD, 2, FF, PP>, 128);    \
    else go(attn_decode_kernel<DD, 1, FF, PP>, 64);                   \
  } while (0)
  const bool parts = fused && ra.part != nullptr;
  if (d == 128) {
    if (parts) {
      if (ra.nparts == 5) DLLM_DEC(128, true, 5);
      else if (ra.nparts == 4) DLLM_DEC(128, true, 4);
      else if (ra.nparts == 3) DLLM_DEC(128, true, 3);   // the 70B qkv (K = 8192, 3 slices)
      else if (ra.nparts == 8) DLLM_DEC(128, true, 8);
      else DLLM_DEC(128, true, -1);
    } else if (fused) DLLM_DEC(128, true, 0); else DLLM_DEC(128, false, 0);
  } else {
    if (parts) DLLM_DEC(64, true, -1); else if (fused) DLLM_DEC(64, true, 0); else DLLM_DEC(64, false, 0);
  }
#undef DLLM_DEC
  DLLM_HIP_CHECK(hipGetLastError());
  if (num_splits > 1) {
    if (d == 128)
      hipLaunchKernelGGL(attn_split_reduce_kernel<128>, dim3(batch * hq), dim3(128), 0, s, (bf16*)out,
                         (const float*)part_o, (const float*)part_ml, num_splits);
    else
      hipLaunchKernelGGL(attn_split_reduce_kernel<64>, dim3(batch * hq), dim3(64), 0, s, (bf16*)out,
                         (const float*)part_o, (const float*)part_ml, num_splits);
    DLLM_HIP_CHECK(hipGetLastError());
  }
}

void paged_attention_decode(uintptr_t out, uintptr_t q, uintptr_t k_cache, uintptr_t v_cache,
                            uintptr_t block_tables, uintptr_t seq_lens, uintptr_t part_o, uintptr_t part_ml,
                            int batch, int hq, int hkv, int d, int block_size, int max_blocks, int num_splits,
                            int split_len, float scale, uintptr_t stream) {
  decode_launch(out, q, k_cache, v_cache, block_tables, seq_lens, part_o, part_ml, batch, hq, hkv, d, block_size,
                max_blocks, num_splits, split_len, scale, RopeArgs{nullptr, nullptr, nullptr, nullptr}, false, stream);
}

// decode with RoPE + KV append fused in: reads the raw qkv projection [B, (hq + 2 hkv) * d]
void paged_attention_decode_rope(uintptr_t out, uintptr_t qkv, uintptr_t positions, uintptr_t cos_sin, uintptr_t slots,
                                 uintptr_t k_cache, uintptr_t v_cache, uintptr_t block_tables, uintptr_t seq_lens,
                                 uintptr_t part_o, uintptr_t part_ml, int batch, int hq, int hkv, int d,
                                 int block_size, int max_blocks, int num_splits, int split_len, float scale,
                                 uintptr_t qkv_part, int qkv_nparts, long qkv_slab, uintptr_t stream) {
  RopeArgs ra{(const bf16*)qkv, (const int32_t*)positions, (const float*)cos_sin, (const int32_t*)slots,
              (const float*)qkv_part, qkv_nparts, qkv_slab};
  decode_launch(out, 0, k_cache, v_cache, block_tables, seq_lens, part_o, part_ml, batch, hq, hkv, d, block_size,
                max_blocks, num_splits, split_len, scale, ra, true, stream);
}

template <int D>
static void launch_prefill(int g, int version, int max_q_len, int batch, int hkv, hipStream_t s, uintptr_t out,
                           uintptr_t q, uintptr_t k_cache, uintptr_t v_cache, uintptr_t bt, uintptr_t cu, uintptr_t sl,
                           int hq, int max_blocks, float sl2, uintptr_t pos, uintptr_t cs, int q_stride) {
  // version 3: the register-tiled kernel, two tiles per wave; 4: the LDS-shared kernel, two tiles per
  // wave; 6: the LDS-shared kernel on 32x32x16 MFMAs, 8 waves x 32 columns (head_dim 128); 7: 6 with
  // the previous tile's P.V overlapping this tile's softmax; 9: 7 persistent (one workgroup per CU)
  const int nt = 2;
  const int rows_per_wg = version >= 6 ? kW32Waves * (32 / g) : kWaves * (16 / g) * nt;
  const dim3 grid((max_q_len + rows_per_wg - 1) / rows_per_wg, hkv, batch);
  // version 9 (persistent): one workgroup per CU, 8 XCDs
  int cus = 0;
  if (version == 9) {
    int dev = 0;
    DLLM_HIP_CHECK(hipGetDevice(&dev));
    DLLM_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cus -= cus % 8;
    DLLM_HOST_CHECK(cus >= 8, "persistent prefill attention: CU count");
  }
#define DLLM_PF(GG)                                                                                         \
  do {                                                                                                      \
    if (version == 9) {                                                                                     \
      if constexpr (D == 128)                                                                               \
        hipLaunchKernelGGL((attn_prefill_w32p_kernel<GG>), dim3(cus), dim3(kW32Waves * 64), 0, s, (bf16*)out, \
                           (const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, (const int32_t*)bt,    \
                           (const int32_t*)cu, (const int32_t*)sl, hq, hkv, max_blocks, sl2,                 \
                           (const int32_t*)pos, (const float*)cs, q_stride, (int)grid.x, batch * hkv);       \
    } else if (version >= 6) {                                                                              \
      if constexpr (D == 128) {                                                                             \
        auto kern = version == 7 ? attn_prefill_w32_kernel<GG, true> : attn_prefill_w32_kernel<GG, false>;   \
        hipLaunchKernelGGL(kern, grid, dim3(kW32Waves * 64), 0, s, (bf16*)out, (const bf16*)q,                \
                           (const bf16*)k_cache, (const bf16*)v_cache, (const int32_t*)bt,                    \
                           (const int32_t*)cu, (const int32_t*)sl, hq, hkv, max_blocks, sl2,                 \
                           (const int32_t*)pos, (const float*)cs, q_stride);                                 \
      }                                                                                                     \
    } else if (version == 4)                                                                                \
      hipLaunchKernelGGL((attn_prefill_lds_kernel<D, GG, 2>), grid, dim3(256), 0, s, (bf16*)out,              \
                         (const bf16*)q, (const bf16*)k_cache, (const bf16*)v_cache, (const int32_t*)bt,      \
                         (const int32_t*)cu, (const int32_t*)sl, hq, hkv, max_blocks, sl2,                   \
                         (const int32_t*)pos, (const float*)cs, q_stride);                                   \
    else                                                                                                    \
      hipLaunchKernelGGL((attn_prefill2_kernel<D, GG, 2>), grid, dim3(256), 0, s, (bf16*)out, (const bf16*)q,  \
                         (const bf16*)k_cache, (const bf16*)v_cache, (const int32_t*)bt, (const int32_t*)cu,   \
                         (const int32_t*)sl, hq, hkv, max_blocks, sl2);                                      \
  } while (0)
  switch (g) {
    case 1: DLLM_PF(1); break;
    case 2: DLLM_PF(2); break;
    case 4: DLLM_PF(4); break;
    case 8: DLLM_PF(8); break;
    case 16: DLLM_PF(16); break;
    default: throw std::runtime_error("prefill attention: GQA group must be 1,2,4,8,16");
  }
#undef DLLM_PF
}

// positions / cos_sin / q_stride: q is the raw qkv projection (row stride q_stride elements) and RoPE
// is applied in the kernel (LDS kernel, version 4); cos_sin = 0: q is [T, hq, D], rotated
void paged_attention_prefill(uintptr_t out, uintptr_t q, uintptr_t k_cache, uintptr_t v_cache,
                             uintptr_t block_tables, uintptr_t cu_seqlens_q, uintptr_t seq_lens, int batch,
                             int hq, int hkv, int d, int block_size, int max_blocks, int max_q_len, float scale,
                             int version, uintptr_t positions, uintptr_t cos_sin, int q_stride, uintptr_t stream) {
  DLLM_HOST_CHECK(block_size == kBS, "paged attention requires block_size 32");
  if (q_stride == 0) q_stride = hq * d;
  DLLM_HOST_CHECK(q_stride >= hq * d && q_stride % 8 == 0, "q row stride");
  DLLM_HOST_CHECK(cos_sin == 0 || positions != 0, "in-kernel RoPE needs positions");
  DLLM_HOST_CHECK(d == 64 || d == 128, "head_dim must be 64 or 128");
  DLLM_HOST_CHECK(hq % hkv == 0, "Hq % Hkv");
  if (batch == 0 || max_q_len == 0) return;
  const int G = hq / hkv;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const float sl2 = scale * 1.4426950408889634f;
  // version (ops.prefill_attn_version): 4 = the LDS-shared kernel (short prompts); 6 / 7 / 9 = the
  // 32x32x16 kernels (9, persistent, by default from 512 query rows; profiles/round6_attention.md);
  // 3 = the register-tiled kernel, which also serves block tables wider than the 32k tokens of
  // block ids the LDS kernels stage
  DLLM_HOST_CHECK(version == 3 || version == 4 || version == 6 || version == 7 || version == 9,
                  "prefill attention version 3, 4, 6, 7 or 9");
  if (version >= 6 && (d != 128 || G > 16)) version = 4;           // the 32x32 kernels: head_dim 128, G | 32
  if (version != 3 && max_blocks > kPfMaxChunks) version = 3;
  DLLM_HOST_CHECK(q_stride == hq * d || version != 3, "in-kernel RoPE / strided q: LDS kernels only (<= 32k context)");
  if (d == 128)
    launch_prefill<128>(G, version, max_q_len, batch, hkv, s, out, q, k_cache, v_cache, block_tables, cu_seqlens_q,
                        seq_lens, hq, max_blocks, sl2, positions, cos_sin, q_stride);
  else
    launch_prefill<64>(G, version, max_q_len, batch, hkv, s, out, q, k_cache, v_cache, block_tables, cu_seqlens_q,
                       seq_lens, hq, max_blocks, sl2, positions, cos_sin, q_stride);
  DLLM_HIP_CHECK(hipGetLastError());
}

}  // namespace dllm
