// Decode GEMM for batch-sized M (128..512): C[M,N] = A[M,K] . B[N,K]^T, bf16 in, f32 accumulate.
//
// Why a second tiled kernel: at M = 256 the decode projections sit on the ridge between weight
// streaming and MFMA (256 FLOP per weight byte).  The 128x128 two-phase kernel (gemm_tiled.hip)
// re-reads every weight tile once per 128-row M tile and drains its single prefetch at every
// barrier; hipBLASLt's 256x128 tile runs the MLP gate|up at ~3.2 TB/s / 0.8 PF in the engine
// (profiles/llama3_8b_b256_kernels_current.md) -- latency-bound at one workgroup per CU.
//
// Structure (gfx950, wave64):
//  * tile BM x 128 x 64 with BM = 256 (128 for M <= 128, 64 for M <= 64): ALL decode rows in one tile, so
//    each weight byte leaves HBM once per step; 512 threads = 8 waves in 4 (M) x 2 (N), wave
//    tile (BM/4) x 64 = (BM/64) x 4 v_mfma_f32_16x16x32_bf16 accumulators;
//  * global -> LDS with global_load_lds_dwordx4 (lane-linear 1 KiB per wave-instruction =
//    8 rows x 128 B), bank-conflict swizzle chunk ^ ((row >> 1) & 7) applied on the per-lane
//    SOURCE address and on the ds_read address (guide rule 21);
//  * THREE LDS buffers (3 x 48 KiB at BM = 256): tiles t+1 and t+2 stay in flight while tile t
//    is multiplied.  One raw s_barrier per K-tile preceded by a COUNTED vmcnt (never 0 in the
//    loop) -- __syncthreads() would drain the LDS-DMA queue (guide "Pipelining across barriers");
//    all LDS lives in one __shared__ array (guide trap 4a);
//  * SwiGLU layout without a weight permutation: the 128 B-tile rows are 16-row groups taken
//    alternately from the gate half and the up half of the fused [2I, K] weight, so the same lane
//    holds gate column j and up column j in neighbouring accumulators and the epilogue writes
//    silu(g) * u directly (no [M, 2I] intermediate, no separate silu_mul launch);
//  * optional split-K: partial slabs (f16 x 2^-6, common.h) in natural column order, reduced by the next op
//    (splitk_add_rms_norm) or by splitk_reduce(_swiglu);
//  * XCD-aware block order (bijective remap): the M tiles and K slices of one N tile run
//    back-to-back on one XCD;
//  * the next tile's LDS-DMA pieces are issued between the MFMAs (pinned with
//    sched_group_barrier): +9 % on the MLP up projection over issuing them after the barrier;
//  * variant bit 32 (the engine default): fragment reads in inline asm with one lgkmcnt wait per
//    MFMA row, substep 1's reads issued under substep 0's MFMAs (hipcc otherwise waits
//    lgkmcnt(0) for all 16 reads before a K-tile's first MFMA): 1-2 % per GEMM, bit-exact.
// Measured and dropped (profiles/wide_gemm.md): BK = 32 with 6 stages and a fragment software
// pipeline (slower: twice the barriers), 4/5 stages at BM = 128, weights pre-tiled into
// contiguous 16 KiB tiles (+0-3 %), setprio, other read/MFMA/VMEM orders.  Ablations at M = 256:
// no LDS reads = same time, no barrier = same time, no staging loads = -21 % -- the loop is bound
// by the load pipeline with a ~50 %-busy MFMA phase behind it.
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace dllm {

typedef int i32x4w __attribute__((ext_vector_type(4)));
typedef int i32x8w __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) void* lds_vptr_w;
typedef __attribute__((address_space(1))) void* glb_vptr_w;

namespace {
constexpr int WBN = 128, WBK = 64;

__device__ __forceinline__ int wswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void wide_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// wait until at most `younger` tiles of G LDS-DMA instructions each are still in flight (younger
// is a compile-time constant after unrolling in the steady state, at most NBUF - 2 <= 6)
template <int G>
__device__ __forceinline__ void wait_tiles(int younger) {
  static_assert(G >= 3 && G <= 9, "G");
  switch (younger <= 0 ? 0 : younger) {
    case 0: wide_vm<0>(); break;
    case 1: wide_vm<G>(); break;
    case 2: wide_vm<2 * G>(); break;
    case 3: wide_vm<3 * G>(); break;
    case 4: wide_vm<4 * G>(); break;
    case 5: wide_vm<5 * G>(); break;
    default: wide_vm<(6 * G < 63 ? 6 * G : 63)>(); break;
  }
}

// Fragment reads the compiler does not count (inline asm), for the SPLITRD K-tile: hipcc waits
// lgkmcnt(0) before the first MFMA of a K-tile whenever LDS-DMA shares the loop, exposing the
// latency of all 16 fragment reads of every wave at once; here each MFMA row waits only for its
// own fragments (`+v` on the wait statement orders the MFMAs after it, guide §5.7 item 1 (ii)).
template <int OFF>
__device__ __forceinline__ bf16x8 lds_frag(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
#define DLLM_LGKM_W1(n) if constexpr (N == n) asm volatile("s_waitcnt lgkmcnt(" #n ")" : "+v"(a));
#define DLLM_LGKM_W5(n) \
  if constexpr (N == n) asm volatile("s_waitcnt lgkmcnt(" #n ")" : "+v"(a), "+v"(b0), "+v"(b1), "+v"(b2), "+v"(b3));
template <int N>
__device__ __forceinline__ void lgkm_wait1(bf16x8& a) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt");
  DLLM_LGKM_W1(0) DLLM_LGKM_W1(1) DLLM_LGKM_W1(2) DLLM_LGKM_W1(3) DLLM_LGKM_W1(4) DLLM_LGKM_W1(5) DLLM_LGKM_W1(6)
  DLLM_LGKM_W1(7) DLLM_LGKM_W1(8) DLLM_LGKM_W1(9) DLLM_LGKM_W1(10) DLLM_LGKM_W1(11) DLLM_LGKM_W1(12)
  DLLM_LGKM_W1(13) DLLM_LGKM_W1(14) DLLM_LGKM_W1(15)
}
template <int N>
__device__ __forceinline__ void lgkm_wait5(bf16x8& a, bf16x8& b0, bf16x8& b1, bf16x8& b2, bf16x8& b3) {
  static_assert(N >= 0 && N <= 15, "lgkmcnt");
  DLLM_LGKM_W5(0) DLLM_LGKM_W5(1) DLLM_LGKM_W5(2) DLLM_LGKM_W5(3) DLLM_LGKM_W5(4) DLLM_LGKM_W5(5) DLLM_LGKM_W5(6)
  DLLM_LGKM_W5(7) DLLM_LGKM_W5(8) DLLM_LGKM_W5(9) DLLM_LGKM_W5(10) DLLM_LGKM_W5(11) DLLM_LGKM_W5(12)
  DLLM_LGKM_W5(13) DLLM_LGKM_W5(14) DLLM_LGKM_W5(15)
}
#undef DLLM_LGKM_W1
#undef DLLM_LGKM_W5
}  // namespace

// B-tile row r (0..127) -> row of the weight matrix.
//   plain:  n0 + r
//   SwiGLU: 16-row group g = r / 16 alternates gate (even g) / up (odd g); output column
//           c = (g / 2) * 16 + r % 16 of this tile's 64 outputs
template <bool SWIGLU>
__device__ __forceinline__ int wide_b_row(int r, int n_t, int half) {
  if (!SWIGLU) return n_t * WBN + r;
  const int g = r >> 4;
  return ((g & 1) ? half : 0) + n_t * 64 + (g >> 1) * 16 + (r & 15);
}

// Large-M (prefill) block order, no K split: groups of 8 row tiles walk the column tiles together,
// so the blocks resident on an XCD share their A row tiles and a band of B in its L2 instead of
// every block streaming its own A tile against one B tile.  b: the XCD-remapped block index.
__device__ __forceinline__ void grouped_tile(int b, int mtiles, int ntiles, int& m_t, int& n_t) {
  const int per = 8 * ntiles, g = b / per, first = g * 8, gsz = min(mtiles - first, 8);
  m_t = first + (b % per) % gsz;
  n_t = (b % per) / gsz;
}

// epilogue shared by both wide kernels: acc[rt][ct] lane holds tile column (lane & 15), rows
// 4 * (lane >> 4) + i of each 16 x 16 fragment
// SCALED (fp8 operands): the accumulator is in quantized units; output = acc * sa[m] * sb[n]
// (per-token activation scale x per-output-channel weight scale), applied before the SwiGLU and
// before a split-K slab store (the cross-slice sum is linear in it).
template <int BM, bool SPLIT, bool SWIGLU, bool SCALED = false>
__device__ __forceinline__ void wide_epilogue(const f32x4 (&acc)[BM / 64][4], bf16* __restrict__ C,
                                              float* __restrict__ P, int M, int N, int m0, int n_t, int split, int wm,
                                              int wn, int lane, const float* __restrict__ sa = nullptr,
                                              const float* __restrict__ sb = nullptr) {
  constexpr int RT = BM / 64;
  const int fr = lane & 15, fq = lane >> 4;
  float sbn[4];
  if constexpr (SCALED) {
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      int n;
      if (SWIGLU && !SPLIT) n = n_t * 64 + (wn * 2 + (ct >> 1)) * 16 + fr + ((ct & 1) ? N / 2 : 0);
      else n = wide_b_row<SWIGLU>(wn * 64 + ct * 16 + fr, n_t, N / 2);
      sbn[ct] = sb[n];
    }
  }
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * (BM / 4) + rt * 16 + 4 * fq + i;
      if (m >= M) continue;
      float v[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) v[ct] = acc[rt][ct][i];
      if constexpr (SCALED) {
        const float s = sa[m];
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) v[ct] *= s * sbn[ct];
      }
      if (SWIGLU && !SPLIT) {
        const int half = N / 2;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int c = n_t * 64 + (wn * 2 + p) * 16 + fr;
          const float g = v[2 * p], u = v[2 * p + 1];
          C[(size_t)m * half + c] = f2bf(silu_f(g) * u);
        }
      } else {
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int n = wide_b_row<SWIGLU>(wn * 64 + ct * 16 + fr, n_t, N / 2);
          if (SPLIT) part_store(P, ((size_t)split * M + m) * N + n, v[ct]);
          else C[(size_t)m * N + n] = f2bf(v[ct]);
        }
      }
    }
  }
}

// The K loop shared by the dense and the grouped (MoE) wide kernels: stages A/B tiles through
// NBUF LDS buffers (LDS-DMA, counted vmcnt, raw barrier) and accumulates acc = A_tile B_tile^T
// over `nt` 64-deep K-tiles.  srcA/srcB: this lane's staging source for K-tile 0.
// VAR & 128 (PF): every staging slot also issues one 4-byte LDS-DMA per lane into a 256-byte
// scratch (`pf_lds`) from `pfB`, a line of the weight tile PFD slots ahead: the weight lines are
// then in the XCD's L2 when their staging pieces go out, so a tile waits for an L2 hit instead of
// an HBM round trip.  One more vm op per slot (counted waits use G + 1); results are unchanged.
constexpr int PFD = 2;
template <int BM, int NBUF, int VAR, bool FP8 = false>
__device__ __forceinline__ void wide_mainloop(bf16* smem, const bf16* const (&srcA)[BM / 64],
                                              const bf16* const (&srcB)[2], int nt, f32x4 (&acc)[BM / 64][4],
                                              int wv, int lane, const bf16* pfB = nullptr, bf16* pf_lds = nullptr) {
  constexpr int AEL = BM * WBK, BEL = WBN * WBK, BUF = AEL + BEL;
  constexpr bool PF = (VAR & 128) != 0;
  constexpr int AI = BM / 64, BI = 2, G0 = AI + BI, G = PF ? G0 + 1 : G0, RT = BM / 64;
  // the L2 prefetch of the weight tile staged PFD slots after this one (clamped: counts stay static)
  auto prefetch = [&](int tile) {
    if constexpr (PF)
      __builtin_amdgcn_global_load_lds((glb_vptr_w)(pfB + min(tile, nt - 1) * WBK), (lds_vptr_w)pf_lds, 4, 0, 0);
  };
  const int wm = wv >> 1, wn = wv & 1;
  // cache policy of the staging loads (aux: 2 = nt): VAR 2 streams the weights nt, VAR 3 both operands
  constexpr int BAUX = (VAR & 7) >= 2 ? 2 : 0, AAUX = (VAR & 7) == 3 ? 2 : 0;
  auto stage = [&](int buf, int t) {
    bf16* base = smem + buf * BUF;
    const int ko = t * WBK;
#pragma unroll
    for (int j = 0; j < AI; ++j)
      __builtin_amdgcn_global_load_lds((glb_vptr_w)(srcA[j] + ko), (lds_vptr_w)(base + (wv * AI + j) * 512), 16, 0,
                                       AAUX);
#pragma unroll
    for (int j = 0; j < BI; ++j)
      __builtin_amdgcn_global_load_lds((glb_vptr_w)(srcB[j] + ko), (lds_vptr_w)(base + AEL + (wv * BI + j) * 512), 16,
                                       0, BAUX);
  };

#pragma unroll
  for (int a = 0; a < RT; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // one glds piece: p < AI -> A rows, else B rows
  auto piece = [&](bf16* base, int ko, int p) {
    if (p < AI)
      __builtin_amdgcn_global_load_lds((glb_vptr_w)(srcA[p] + ko), (lds_vptr_w)(base + (wv * AI + p) * 512), 16, 0,
                                       AAUX);
    else
      __builtin_amdgcn_global_load_lds((glb_vptr_w)(srcB[p - AI] + ko),
                                       (lds_vptr_w)(base + AEL + (wv * BI + p - AI) * 512), 16, 0, BAUX);
  };
  // one K-tile of MFMAs from buffer `cur`; with STG the next tile's G LDS-DMA pieces are issued
  // in between the MFMAs (each glds costs ~60-185 issue cycles: issued back to back after the
  // barrier they idle the MFMA pipe -- spread out, they hide under MFMA execution)
  auto ktile = [&](int cur, bf16* dst, int ko, auto stg) {
    constexpr bool STG = decltype(stg)::value;
    const bf16* sa = smem + cur * BUF;
    const bf16* sb = sa + AEL;
    bf16x8 fa[2][RT], fb[2][4];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        const int row = wm * (BM / 4) + rt * 16 + fr;
        fa[s][rt] = *reinterpret_cast<const bf16x8*>(sa + row * WBK + wswz(row, 4 * s + fq) * 8);
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int row = wn * 64 + ct * 16 + fr;
        fb[s][ct] = *reinterpret_cast<const bf16x8*>(sb + row * WBK + wswz(row, 4 * s + fq) * 8);
      }
    }
    constexpr int NMF = 2 * RT * 4;
    constexpr int EVERY = NMF / (G0 + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt)
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][rt], fb[s][ct], acc[rt][ct], 0, 0, 0);
          if constexpr (STG) {
            const int i = (s * RT + rt) * 4 + ct + 1;
            if (i % EVERY == 0 && i / EVERY <= G0) piece(dst, ko, i / EVERY - 1);
          }
        }
    if constexpr (STG) {
      // pin the interleave: 8 LDS reads of substep 0, then (EVERY MFMAs, 1 VMEM) x G0, rest
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (RT + 4), 0);
#pragma unroll
      for (int g = 0; g < G0; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, EVERY, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NMF - G0 * EVERY, 0);
    }
  };

  // SPLITRD (VAR & 32): the same K-tile with asm fragment reads and per-row lgkmcnt waits:
  // substep 0's reads, its first MFMA row, substep 1's reads (overlapping substep 0's MFMAs),
  // then each row waits only for its own A fragment; the G staging pieces are spread over rows.
  // Per-lane LDS byte offsets: fragment (rt | ct) of substep s sits at base_s + (rt | ct) * 2 KiB.
  const uint32_t lds0 = (uint32_t)(size_t)(lds_vptr_w)smem;
  uint32_t aoff[2], boff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int ra = wm * (BM / 4) + fr, rb = wn * 64 + fr;
    aoff[s] = (uint32_t)(ra * WBK + wswz(ra, 4 * s + fq) * 8) * 2;
    boff[s] = (uint32_t)(AEL + rb * WBK + wswz(rb, 4 * s + fq) * 8) * 2;
  }
  auto ktile_sr = [&](int cur, bf16* dst, int ko, auto stg) {
    constexpr bool STG = decltype(stg)::value;
    constexpr int ROWS = 2 * RT;
    const uint32_t base = lds0 + (uint32_t)(cur * BUF * 2);
    bf16x8 fa[2][RT], fb[2][4];
    auto reads = [&](int s) {
      const uint32_t ab = base + aoff[s], bb = base + boff[s];
      fb[s][0] = lds_frag<0>(bb);
      fb[s][1] = lds_frag<2048>(bb);
      fb[s][2] = lds_frag<4096>(bb);
      fb[s][3] = lds_frag<6144>(bb);
      fa[s][0] = lds_frag<0>(ab);
      if constexpr (RT > 1) fa[s][1] = lds_frag<2048>(ab);
      if constexpr (RT > 2) fa[s][2] = lds_frag<4096>(ab);
      if constexpr (RT > 3) fa[s][3] = lds_frag<6144>(ab);
    };
    auto row = [&](int s, int rt) {
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
        acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][rt], fb[s][ct], acc[rt][ct], 0, 0, 0);
      if constexpr (STG) {
        const int r = s * RT + rt;
#pragma unroll
        for (int p = 0; p < G0; ++p)
          if ((p * ROWS) / G0 == r) piece(dst, ko, p);
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    reads(0);
    lgkm_wait5<RT - 1>(fa[0][0], fb[0][0], fb[0][1], fb[0][2], fb[0][3]);
    __builtin_amdgcn_sched_barrier(0);
    row(0, 0);
    reads(1);
    __builtin_amdgcn_sched_barrier(0);
    // rows 1.. of substep 0: younger outstanding reads = the rest of fa[0] + all of substep 1
    if constexpr (RT > 1) { lgkm_wait1<RT - 2 + RT + 4>(fa[0][1]); __builtin_amdgcn_sched_barrier(0); row(0, 1); }
    if constexpr (RT > 2) { lgkm_wait1<RT - 3 + RT + 4>(fa[0][2]); __builtin_amdgcn_sched_barrier(0); row(0, 2); }
    if constexpr (RT > 3) { lgkm_wait1<RT - 4 + RT + 4>(fa[0][3]); __builtin_amdgcn_sched_barrier(0); row(0, 3); }
    lgkm_wait5<RT - 1>(fa[1][0], fb[1][0], fb[1][1], fb[1][2], fb[1][3]);
    __builtin_amdgcn_sched_barrier(0);
    row(1, 0);
    if constexpr (RT > 1) { lgkm_wait1<RT - 2>(fa[1][1]); __builtin_amdgcn_sched_barrier(0); row(1, 1); }
    if constexpr (RT > 2) { lgkm_wait1<RT - 3>(fa[1][2]); __builtin_amdgcn_sched_barrier(0); row(1, 2); }
    if constexpr (RT > 3) { lgkm_wait1<RT - 4>(fa[1][3]); __builtin_amdgcn_sched_barrier(0); row(1, 3); }
  };
  // FP8: the same 128-byte LDS rows hold 128 e4m3 values of K; lane group fq's fragment is chunks
  // 2fq and 2fq + 1 (k = 32 fq .. 32 fq + 31, the same k map for A and B), one block-scaled
  // v_mfma_scale_f32_16x16x128_f8f6f4 per (row, column) fragment pair and K-tile (unit E8M0 scales:
  // the real per-token / per-channel scales are applied in the epilogue).  Same cycles per K-tile
  // as the bf16 loop at twice the K: half the K-tiles, half the staging instructions per FLOP.
  auto ktile8 = [&](int cur, bf16* dst, int ko, auto stg) {
    constexpr bool STG = decltype(stg)::value;
    const bf16* sa = smem + cur * BUF;
    const bf16* sb = sa + AEL;
    i32x8w fa[RT], fb[4];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      const int row = wm * (BM / 4) + rt * 16 + fr;
      const i32x4w lo = *reinterpret_cast<const i32x4w*>(sa + row * WBK + wswz(row, 2 * fq) * 8);
      const i32x4w hi = *reinterpret_cast<const i32x4w*>(sa + row * WBK + wswz(row, 2 * fq + 1) * 8);
      fa[rt] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int row = wn * 64 + ct * 16 + fr;
      const i32x4w lo = *reinterpret_cast<const i32x4w*>(sb + row * WBK + wswz(row, 2 * fq) * 8);
      const i32x4w hi = *reinterpret_cast<const i32x4w*>(sb + row * WBK + wswz(row, 2 * fq + 1) * 8);
      fb[ct] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    }
    constexpr int NMF = RT * 4;
    constexpr int EVERY = NMF / (G0 + 1) > 0 ? NMF / (G0 + 1) : 1;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        acc[rt][ct] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fa[rt], fb[ct], acc[rt][ct], 0, 0, 0, 127, 0, 127);
        if constexpr (STG) {
          const int i = rt * 4 + ct + 1;
          if (i % EVERY == 0 && i / EVERY <= G0) piece(dst, ko, i / EVERY - 1);
        }
      }
    if constexpr (STG) {
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * (RT + 4), 0);
#pragma unroll
      for (int g = 0; g < G0; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x008, EVERY, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, NMF - G0 * EVERY, 0);
    }
  };
  constexpr bool SPLITRD = (VAR & 32) != 0 && RT <= 4 && !FP8;

  if (nt > 0) {
#pragma unroll
    for (int p = 0; p < NBUF - 1; ++p)
      if (p < nt) {
        prefetch(p + PFD);
        stage(p, p);
      }
    int cur = 0;
    int t = 0;
    // steady state: tile t + NBUF - 1 exists, NBUF - 2 younger tiles stay in flight
    for (; t + NBUF - 1 < nt; ++t) {
      wait_tiles<G>(NBUF - 2);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      prefetch(t + NBUF - 1 + PFD);
      // buffer (t-1) % NBUF was last read in iteration t-1, which every wave finished before
      // this barrier: refill it with tile t + NBUF - 1
      const int nb = cur == 0 ? NBUF - 1 : cur - 1;
      if constexpr (FP8) {
        ktile8(cur, smem + nb * BUF, (t + NBUF - 1) * WBK, std::true_type{});
      } else if constexpr (SPLITRD) {
        ktile_sr(cur, smem + nb * BUF, (t + NBUF - 1) * WBK, std::true_type{});
      } else if constexpr ((VAR & 7) == 0) {
        stage(nb, t + NBUF - 1);
        ktile(cur, smem, 0, std::false_type{});
      } else {
        ktile(cur, smem + nb * BUF, (t + NBUF - 1) * WBK, std::true_type{});
      }
      cur = cur == NBUF - 1 ? 0 : cur + 1;
    }
    // drain: no more tiles to stage
    for (; t < nt; ++t) {
      wait_tiles<G>(nt - 1 - t);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if constexpr (FP8) ktile8(cur, smem, 0, std::false_type{});
      else if constexpr (SPLITRD) ktile_sr(cur, smem, 0, std::false_type{});
      else ktile(cur, smem, 0, std::false_type{});
      cur = cur == NBUF - 1 ? 0 : cur + 1;
    }
  }

}

template <int BM, bool SPLIT, bool SWIGLU, int NBUF, int VAR>
__global__ void __launch_bounds__(512, 1) gemm_wide_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                           int K, int kt_per_split, int nsplit) {
  constexpr int AEL = BM * WBK, BEL = WBN * WBK, BUF = AEL + BEL;   // bf16 elements
  constexpr int AI = BM / 64;                 // A glds instructions per thread per tile
  constexpr int BI = 2;                       // B glds instructions per thread per tile
  constexpr int G = AI + BI;                  // glds per thread per tile (vmcnt unit)
  constexpr int RT = BM / 64;                 // 16-row fragments per wave in M
  constexpr int PFL = (VAR & 128) ? 128 : 0;  // L2-prefetch scratch (bf16 elements), same LDS array
  static_assert(NBUF >= 3 && (NBUF * BUF + PFL) * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 smem[NBUF * BUF + PFL];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int mtiles = (M + BM - 1) / BM;
  const int ntiles = SWIGLU ? (N / 2) / 64 : N / WBN;
  const int total = gridDim.x;
  // bijective XCD remap: blocks b with b % 8 == x run on XCD x; give XCD x a contiguous run
  int b = blockIdx.x;
  {
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  int m_t = b % mtiles, rest = b / mtiles;
  int split = rest % nsplit, n_t = rest / nsplit;
  if constexpr ((VAR & 64) != 0) {          // prefill M, no K split (grouped_tile)
    grouped_tile(b, mtiles, ntiles, m_t, n_t);
    split = 0;
  }
  const int m0 = m_t * BM;
  const int kt0 = split * kt_per_split;
  // ablations (timing only, wrong results): VAR & 16 skips the K loop (launch + epilogue cost),
  // VAR & 8 skips the epilogue stores (kept behind a never-true runtime test so the MFMAs stay)
  const int nt = (VAR & 16) ? 0 : max(0, min(K / WBK, kt0 + kt_per_split) - kt0);

  // per-lane staging sources: instruction i covers tile rows 8i .. 8i+7, lane -> (row, chunk)
  const bf16* srcA[AI];
  const bf16* srcB[BI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int i = wv * AI + j;
    const int r = 8 * i + (lane >> 3);
    srcA[j] = A + (size_t)min(m0 + r, M - 1) * K + (size_t)kt0 * WBK + wswz(r, lane & 7) * 8;
  }
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int i = wv * BI + j;
    const int r = 8 * i + (lane >> 3);
    srcB[j] = B + (size_t)wide_b_row<SWIGLU>(r, n_t, N / 2) * K + (size_t)kt0 * WBK + wswz(r, lane & 7) * 8;
  }
  // PF: lanes l and l + 16k of wave w touch weight row 16 w + (l & 15) of the tile: 128 lines per K-tile
  const bf16* pfB = B + (size_t)wide_b_row<SWIGLU>(16 * wv + (lane & 15), n_t, N / 2) * K + (size_t)kt0 * WBK;
  f32x4 acc[RT][4];
  wide_mainloop<BM, NBUF, VAR>(smem, srcA, srcB, nt, acc, wv, lane, pfB, smem + NBUF * BUF);
  if (VAR & 8) return;
  wide_epilogue<BM, SPLIT, SWIGLU>(acc, C, P, M, N, m0, n_t, split, wm, wn, lane);
}

// FP8 (W8A8) variant: A [M, K] and B [N, K] OCP e4m3 bytes, per-row scales sa [M] (dynamic,
// per token: ops/quant) and sb [N] (per output channel, at load time).  Staging is the bf16 kernel's
// byte for byte: a 128 x 128-byte K-tile is 128 K of fp8, addressed as 64 bf16-sized units.
template <int BM, bool SPLIT, bool SWIGLU, int NBUF, int VAR>
__global__ void __launch_bounds__(512, 1) gemm_wide_fp8_kernel(const uint8_t* __restrict__ A8,
                                                               const uint8_t* __restrict__ B8, const float* __restrict__ sa,
                                                               const float* __restrict__ sb, bf16* __restrict__ C,
                                                               float* __restrict__ P, int M, int N, int K,
                                                               int kt_per_split, int nsplit) {
  constexpr int AEL = BM * WBK, BEL = WBN * WBK, BUF = AEL + BEL;   // 2-byte units
  constexpr int AI = BM / 64, BI = 2, RT = BM / 64;
  static_assert(NBUF >= 3 && NBUF * BUF * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 smem[NBUF * BUF];
  const bf16* A = reinterpret_cast<const bf16*>(A8);
  const bf16* B = reinterpret_cast<const bf16*>(B8);
  const int KU = K / 2;                       // row length in 2-byte units

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int mtiles = (M + BM - 1) / BM;
  const int total = gridDim.x;
  int b = blockIdx.x;
  {
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  int m_t = b % mtiles, rest = b / mtiles;
  int split = rest % nsplit, n_t = rest / nsplit;
  if constexpr ((VAR & 64) != 0) {          // prefill M, no K split (column tiles: N / 128 both ways)
    grouped_tile(b, mtiles, N / WBN, m_t, n_t);
    split = 0;
  }
  const int m0 = m_t * BM;
  const int kt0 = split * kt_per_split;
  const int nt = max(0, min(KU / WBK, kt0 + kt_per_split) - kt0);
  const bf16* srcA[AI];
  const bf16* srcB[BI];
#pragma unroll
  for (int j = 0; j < AI; ++j) {
    const int r = 8 * (wv * AI + j) + (lane >> 3);
    srcA[j] = A + (size_t)min(m0 + r, M - 1) * KU + (size_t)kt0 * WBK + wswz(r, lane & 7) * 8;
  }
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int r = 8 * (wv * BI + j) + (lane >> 3);
    srcB[j] = B + (size_t)wide_b_row<SWIGLU>(r, n_t, N / 2) * KU + (size_t)kt0 * WBK + wswz(r, lane & 7) * 8;
  }
  f32x4 acc[RT][4];
  wide_mainloop<BM, NBUF, VAR, true>(smem, srcA, srcB, nt, acc, wv, lane);
  wide_epilogue<BM, SPLIT, SWIGLU, true>(acc, C, P, M, N, m0, n_t, split, wm, wn, lane, sa, sb);
}

// ---------------------------------------------------------------------------------------------
// Grouped (MoE) wide GEMM: grid (column tiles, experts).  Expert e owns rows [offsets[e],
// offsets[e] + counts[e]) of the expert-sorted slot space; its A rows are gathered through
// `gather` (slot -> token row of X; null = slot rows of X), its weight is W[e] ([N, K], SwiGLU:
// [2I, K] with the alternating gate/up row groups of the dense kernel).  The row tile is picked
// per expert from its count (workgroup-uniform): 64 rows up to 64, else 128-row chunks.  This is
// the decode regime of Mixtral at B >= 128 (32-128 rows per expert), where the weight-streaming
// grouped kernel (moe.hip) runs its MFMAs at a fraction of the rate.
// ---------------------------------------------------------------------------------------------
template <int BM, bool SWIGLU, int VAR, bool FP8 = false, int NBUF = 3>
__device__ __forceinline__ void moe_wide_rows(bf16* smem, bf16* __restrict__ Y, const bf16* __restrict__ X,
                                              const int* __restrict__ gather, const bf16* __restrict__ We, int cnt,
                                              int off, int N, int K, int n_t, int wv, int lane,
                                              const float* __restrict__ sa = nullptr,
                                              const float* __restrict__ sb = nullptr) {
  // FP8: X / We hold e4m3 bytes addressed in 2-byte units (K / 2 per row); sa: per-slot activation
  // scales (slot order), sb: this expert's per-channel weight scales
  constexpr int AI = BM / 64, BI = 2, RT = BM / 64;
  const int KU = FP8 ? K / 2 : K;
  const int wm = wv >> 1, wn = wv & 1;
  const int ldy = SWIGLU ? N / 2 : N;
  for (int r0 = 0; r0 < cnt; r0 += BM) {
    const int rows = min(BM, cnt - r0);
    const bf16* srcA[AI];
    const bf16* srcB[BI];
#pragma unroll
    for (int j = 0; j < AI; ++j) {
      const int r = 8 * (wv * AI + j) + (lane >> 3);
      const int slot = off + r0 + min(r, rows - 1);
      const int src = gather ? gather[slot] : slot;
      srcA[j] = X + (size_t)src * KU + wswz(r, lane & 7) * 8;
    }
#pragma unroll
    for (int j = 0; j < BI; ++j) {
      const int r = 8 * (wv * BI + j) + (lane >> 3);
      srcB[j] = We + (size_t)wide_b_row<SWIGLU>(r, n_t, N / 2) * KU + wswz(r, lane & 7) * 8;
    }
    f32x4 acc[RT][4];
    wide_mainloop<BM, NBUF, VAR, FP8>(smem, srcA, srcB, KU / WBK, acc, wv, lane);
    wide_epilogue<BM, false, SWIGLU, FP8>(acc, Y + (size_t)(off + r0) * ldy, nullptr, rows, N, 0, n_t, 0, wm, wn,
                                          lane, FP8 ? sa + off + r0 : nullptr, sb);
    __syncthreads();   // the next chunk's prologue refills buffers other waves may still read
  }
}

// Ring depth (moe_wide_nbuf): at 32-128 rows per expert the K loop is bound by weight bytes in
// flight, not by the MFMAs (a 64-row K-tile is 128 MFMA cycles per SIMD against ~1 us of HBM
// latency), so the ring is as deep as the 160 KiB of LDS allow: 64-row tiles 6 x 24 KiB (five
// K-tiles in flight), 128-row tiles 5 x 32 KiB (four).  NBUF_SEL 0 = the 3-slot ring (A/B runs).
constexpr int MOE_LDS = 5 * (128 + WBN) * WBK;    // bf16 elements (160 KiB)
template <int BM, int NBUF_SEL>
constexpr int moe_nbuf() {
  return NBUF_SEL == 0 ? 3 : (BM == 64 ? 6 : 5);
}

template <bool SWIGLU, bool FP8 = false, int NBUF_SEL = 1>
__global__ void __launch_bounds__(512, 1) moe_wide_kernel(bf16* __restrict__ Y, const bf16* __restrict__ X,
                                                          const int* __restrict__ gather, const bf16* __restrict__ W,
                                                          const int* __restrict__ counts,
                                                          const int* __restrict__ offsets, int N, int K, int nt,
                                                          const float* __restrict__ sa = nullptr,
                                                          const float* __restrict__ wscale = nullptr) {
  static_assert(moe_nbuf<64, NBUF_SEL>() * (64 + WBN) * WBK <= MOE_LDS &&
                moe_nbuf<128, NBUF_SEL>() * (128 + WBN) * WBK <= MOE_LDS, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 smem[MOE_LDS];
  const int e = blockIdx.y;
  const int cnt = counts[e];
  if (cnt == 0) return;                       // uniform across the workgroup
  const int off = offsets[e];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bf16* We = W + (size_t)e * N * (FP8 ? K / 2 : K);
  const float* sb = FP8 ? wscale + (size_t)e * N : nullptr;
  constexpr int NB64 = moe_nbuf<64, NBUF_SEL>(), NB128 = moe_nbuf<128, NBUF_SEL>();
  // an expert's weight tile is read once when its rows fit one row tile: stream it nt (variant 2);
  // with several row chunks the re-reads should hit the caches (default policy)
  if (cnt <= 64) {
    if (nt) moe_wide_rows<64, SWIGLU, 2, FP8, NB64>(smem, Y, X, gather, We, cnt, off, N, K, blockIdx.x, wv, lane, sa, sb);
    else moe_wide_rows<64, SWIGLU, 1, FP8, NB64>(smem, Y, X, gather, We, cnt, off, N, K, blockIdx.x, wv, lane, sa, sb);
  } else if (cnt <= 128 && nt) {
    moe_wide_rows<128, SWIGLU, 2, FP8, NB128>(smem, Y, X, gather, We, cnt, off, N, K, blockIdx.x, wv, lane, sa, sb);
  } else {
    moe_wide_rows<128, SWIGLU, 1, FP8, NB128>(smem, Y, X, gather, We, cnt, off, N, K, blockIdx.x, wv, lane, sa, sb);
  }
}

// mode 1 (SwiGLU): W [E, 2I, K] -> Y [slots, I]; mode 0: W [E, N, K] -> Y [slots, N]
void moe_wide_gemm(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                   int E, int N, int K, int mode, uintptr_t stream) {
  DLLM_HOST_CHECK(E >= 1, "experts >= 1");
  DLLM_HOST_CHECK(K % WBK == 0, "K must be a multiple of 64");
  DLLM_HOST_CHECK(N % 128 == 0, "N must be a multiple of 128");
  // mode bit 2: the 3-slot ring instead of the deep one (A/B runs)
  const bool shallow = (mode & 4) != 0;
  mode &= 3;
  DLLM_HOST_CHECK(mode == 0 || mode == 1, "mode");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ntiles = mode == 1 ? (N / 2) / 64 : N / WBN;
  constexpr int nt = 1;   // expert weights are read once per step: nontemporal
#define DLLM_MOE_GO(SW_, SEL_)                                                                                   \
  hipLaunchKernelGGL((moe_wide_kernel<SW_, false, SEL_>), dim3(ntiles, E), dim3(512), 0, s, (bf16*)y,            \
                     (const bf16*)x, (const int*)gather, (const bf16*)w, (const int*)counts, (const int*)offsets, N, \
                     K, nt, (const float*)nullptr, (const float*)nullptr)
  if (mode == 1) { if (shallow) DLLM_MOE_GO(true, 0); else DLLM_MOE_GO(true, 1); }
  else { if (shallow) DLLM_MOE_GO(false, 0); else DLLM_MOE_GO(false, 1); }
#undef DLLM_MOE_GO
  DLLM_HIP_CHECK(hipGetLastError());
}

// FP8 experts: X e4m3 [tokens or slots, K] (+ gather), W e4m3 [E, N, K] with per-channel scales
// wscale [E, N], sa: per-slot activation scales in slot order.  K % 128 == 0.
void moe_wide_gemm_fp8(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                       int E, int N, int K, int mode, uintptr_t sa, uintptr_t wscale, uintptr_t stream) {
  DLLM_HOST_CHECK(E >= 1, "experts >= 1");
  DLLM_HOST_CHECK(K % 128 == 0, "fp8 K must be a multiple of 128");
  DLLM_HOST_CHECK(N % 128 == 0, "N must be a multiple of 128");
  DLLM_HOST_CHECK(mode == 0 || mode == 1, "mode");
  DLLM_HOST_CHECK(sa != 0 && wscale != 0, "fp8 grouped GEMM needs both scale vectors");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ntiles = mode == 1 ? (N / 2) / 64 : N / WBN;
  constexpr int nt = 1;   // expert weights are read once per step: nontemporal
  if (mode == 1)
    hipLaunchKernelGGL((moe_wide_kernel<true, true>), dim3(ntiles, E), dim3(512), 0, s, (bf16*)y, (const bf16*)x,
                       (const int*)gather, (const bf16*)w, (const int*)counts, (const int*)offsets, N, K, nt,
                       (const float*)sa, (const float*)wscale);
  else
    hipLaunchKernelGGL((moe_wide_kernel<false, true>), dim3(ntiles, E), dim3(512), 0, s, (bf16*)y, (const bf16*)x,
                       (const int*)gather, (const bf16*)w, (const int*)counts, (const int*)offsets, N, K, nt,
                       (const float*)sa, (const float*)wscale);
  DLLM_HIP_CHECK(hipGetLastError());
}

static int wide_bm(int M) {
  if (M <= 64) return 64;
  if (M <= 128) return 128;
  if (M <= 192) return 192;
  if (M <= 256) return 256;
  if (M <= 384) return 192;
  return 256;
}

// mode 0: C = A B^T;  mode 1: SwiGLU, C[M, N/2] = silu(A Bg^T) * (A Bu^T) with B = [Bg; Bu];
// mode 2: leave split-K partial slabs in ws (no reduce; S > 1 required).
// Returns the effective number of K slices S (the partial slabs a deferred reduce must sum).
int gemm_wide(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
              int mode, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(K % WBK == 0, "K must be a multiple of 64");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  const bool swiglu = mode == 1;
  DLLM_HOST_CHECK(swiglu ? (N % 128 == 0) : (N % WBN == 0), "N must be a multiple of 128");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  // variant bits 8..: optional row tile override (64 / 128 / 192 / 256), 0 = wide_bm(M)
  const int bm_force = variant >> 8;
  variant &= 0xff;
  DLLM_HOST_CHECK(bm_force == 0 || bm_force == 64 || bm_force == 128 || bm_force == 192 || bm_force == 256,
                  "row tile override must be 64, 128, 192 or 256");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ktiles = K / WBK;
  const int kts = (ktiles + splits - 1) / splits;
  const int S = (ktiles + kts - 1) / kts;
  DLLM_HOST_CHECK(mode != 2 || S > 1, "mode 2 needs a K split");
  // row tile: the smallest of 64 / 128 / 192 / 256 that covers M, or 192 for 256 < M <= 384
  // (two 192-row tiles instead of a half-empty second 256-row tile)
  const int BM = bm_force ? bm_force : wide_bm(M);
  const int mtiles = (M + BM - 1) / BM;
  const int ntiles = swiglu ? (N / 2) / 64 : N / WBN;
  const long grid = (long)ntiles * mtiles * S;
  DLLM_HOST_CHECK(grid >= 1 && grid < (1L << 31), "grid");
  if (S > 1) DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");

  // weights nt (variant 2) where the grid has no K split: -3..-5 % on the MLP up projection from
  // cold caches; on the split-K grids nt costs up to +25 % at M = 128 (profiles/wide_gemm.md)
  // (variant 4 = variant 1 everywhere, for A/B runs)
  // variant | 32: per-row fragment waits (SPLITRD in wide_mainloop; the engine default);
  // ablations (A/B timing only): variant | 8 = no epilogue stores, | 16 = no K loop
  const int abl = variant & 56;
  const bool grp = (variant & 64) != 0 && S == 1;   // grouped row-tile order (large M)
  const bool pf = (variant & 128) != 0;            // L2 prefetch of the weight tile (wide_mainloop PF)
  variant &= 7;
  if (variant == 1 && S == 1) variant = grp ? 1 : 2;
  else if (variant == 4) variant = 1;
#define DLLM_WIDE_GO3(BM_, SPLIT_, SW_, V_)                                                                      \
  hipLaunchKernelGGL((gemm_wide_kernel<BM_, SPLIT_, SW_, 3, V_>), dim3((unsigned)grid), dim3(512), 0, s,          \
                     (const bf16*)a, (const bf16*)b, (bf16*)c, (float*)ws, M, N, K, kts, S)
#define DLLM_WIDE_GO(BM_, SPLIT_, SW_)                                                                          \
  do {                                                                                                         \
    if (abl == 8) { if (variant == 2) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 10); else DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 9); } \
    else if (abl == 16) { if (variant == 2) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 18); else DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 17); } \
    else if (pf && abl == 32) { if (variant == 2) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 162); else DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 161); } \
    else if (pf) { if (variant == 2) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 130); else DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 129); } \
    else if (abl == 32) { if (variant == 2) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 34); else DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 33); } \
    else if (grp && !SPLIT_) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 65);                                              \
    else if (variant == 0) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 0);                                                 \
    else if (variant == 2) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 2);                                                 \
    else if (variant == 3) DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 3);                                                 \
    else DLLM_WIDE_GO3(BM_, SPLIT_, SW_, 1);                                                                   \
  } while (0)
  if (S == 1) {
    if (BM == 64) { if (swiglu) DLLM_WIDE_GO(64, false, true); else DLLM_WIDE_GO(64, false, false); }
    else if (BM == 128) { if (swiglu) DLLM_WIDE_GO(128, false, true); else DLLM_WIDE_GO(128, false, false); }
    else if (BM == 192) { if (swiglu) DLLM_WIDE_GO(192, false, true); else DLLM_WIDE_GO(192, false, false); }
    else { if (swiglu) DLLM_WIDE_GO(256, false, true); else DLLM_WIDE_GO(256, false, false); }
    DLLM_HIP_CHECK(hipGetLastError());
    return 1;
  }
  if (BM == 64) { if (swiglu) DLLM_WIDE_GO(64, true, true); else DLLM_WIDE_GO(64, true, false); }
  else if (BM == 128) { if (swiglu) DLLM_WIDE_GO(128, true, true); else DLLM_WIDE_GO(128, true, false); }
  else if (BM == 192) { if (swiglu) DLLM_WIDE_GO(192, true, true); else DLLM_WIDE_GO(192, true, false); }
  else { if (swiglu) DLLM_WIDE_GO(256, true, true); else DLLM_WIDE_GO(256, true, false); }
#undef DLLM_WIDE_GO
#undef DLLM_WIDE_GO3
  DLLM_HIP_CHECK(hipGetLastError());
  if (mode == 2) return S;
  splitk_reduce_ex(c, ws, 0, S, M, N, swiglu ? 1 : 0, stream);
  return S;
}

// FP8 W8A8 wide GEMM: modes as gemm_wide; K in elements (= bytes), multiple of 128.
int gemm_wide_fp8(uintptr_t c, uintptr_t a, uintptr_t a_scale, uintptr_t b, uintptr_t b_scale, uintptr_t ws,
                  long ws_floats, int M, int N, int K, int splits, int mode, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(K % 128 == 0, "fp8 K must be a multiple of 128");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  DLLM_HOST_CHECK(a_scale != 0 && b_scale != 0, "fp8 GEMM needs both scale vectors");
  const bool swiglu = mode == 1;
  DLLM_HOST_CHECK(N % 128 == 0, "N must be a multiple of 128");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  const int bm_force = variant >> 8;
  variant &= 0xff;
  DLLM_HOST_CHECK(bm_force == 0 || bm_force == 64 || bm_force == 128 || bm_force == 192 || bm_force == 256,
                  "row tile override must be 64, 128, 192 or 256");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ktiles = K / 128;
  const int kts = (ktiles + splits - 1) / splits;
  const int S = (ktiles + kts - 1) / kts;
  DLLM_HOST_CHECK(mode != 2 || S > 1, "mode 2 needs a K split");
  const int BM = bm_force ? bm_force : wide_bm(M);
  const int mtiles = (M + BM - 1) / BM;
  const int ntiles = swiglu ? (N / 2) / 64 : N / WBN;
  const long grid = (long)ntiles * mtiles * S;
  DLLM_HOST_CHECK(grid >= 1 && grid < (1L << 31), "grid");
  if (S > 1) DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  // weights nt where the grid has no K split (as the bf16 kernel's variant 1); variant | 64: grouped
  // row-tile order for large M (no K split)
  const bool nt = (variant & 7) != 4 && S == 1;
  const bool grp = (variant & 64) != 0 && S == 1 && !nt;
#define DLLM_F8_GO3(BM_, SPLIT_, SW_, V_)                                                                   \
  hipLaunchKernelGGL((gemm_wide_fp8_kernel<BM_, SPLIT_, SW_, 3, V_>), dim3((unsigned)grid), dim3(512), 0, s,  \
                     (const uint8_t*)a, (const uint8_t*)b, (const float*)a_scale, (const float*)b_scale,      \
                     (bf16*)c, (float*)ws, M, N, K, kts, S)
#define DLLM_F8_GO(BM_, SPLIT_, SW_)                                   \
  do {                                                                \
    if (nt) DLLM_F8_GO3(BM_, SPLIT_, SW_, 2);                          \
    else if (grp && !SPLIT_) DLLM_F8_GO3(BM_, SPLIT_, SW_, 65);          \
    else DLLM_F8_GO3(BM_, SPLIT_, SW_, 1);                              \
  } while (0)
  if (S == 1) {
    if (BM == 64) { if (swiglu) DLLM_F8_GO(64, false, true); else DLLM_F8_GO(64, false, false); }
    else if (BM == 128) { if (swiglu) DLLM_F8_GO(128, false, true); else DLLM_F8_GO(128, false, false); }
    else if (BM == 192) { if (swiglu) DLLM_F8_GO(192, false, true); else DLLM_F8_GO(192, false, false); }
    else { if (swiglu) DLLM_F8_GO(256, false, true); else DLLM_F8_GO(256, false, false); }
    DLLM_HIP_CHECK(hipGetLastError());
    return 1;
  }
  if (BM == 64) { if (swiglu) DLLM_F8_GO(64, true, true); else DLLM_F8_GO(64, true, false); }
  else if (BM == 128) { if (swiglu) DLLM_F8_GO(128, true, true); else DLLM_F8_GO(128, true, false); }
  else if (BM == 192) { if (swiglu) DLLM_F8_GO(192, true, true); else DLLM_F8_GO(192, true, false); }
  else { if (swiglu) DLLM_F8_GO(256, true, true); else DLLM_F8_GO(256, true, false); }
#undef DLLM_F8_GO
#undef DLLM_F8_GO3
  DLLM_HIP_CHECK(hipGetLastError());
  if (mode == 2) return S;
  splitk_reduce_ex(c, ws, 0, S, M, N, swiglu ? 1 : 0, stream);
  return S;
}

}  // namespace dllm
