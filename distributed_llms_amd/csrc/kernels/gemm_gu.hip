// Decode MLP gate|up + SwiGLU at 192 < M <= 256 with every CU busy:
//   C[M, I] = silu(A Wg^T) * (A Wu^T),  W = [Wg; Wu] ([2I, K], nn.Linear layout), bf16 in, f32 acc.
//
// Why a kernel of its own: at M = 256 the SwiGLU-fused gemm_wide tile (256 rows x 64 outputs) gives
// Llama-3-8B (I = 14336) 224 workgroups -- 32 of the 256 CUs idle -- and this projection is close to
// MFMA-bound at that M (60 GFLOP against 235 MB of weights; the no-staging ablation of gemm_wide
// still takes 52 of its 66 us, profiles/wide_gemm.md).  Here a workgroup owns 56 outputs
// (I / 56 = 256 workgroups for I = 14336, 512 for the 70B's 28672), so the MFMA work spreads over
// all CUs.
//
// Structure (gfx950, wave64, 8 waves = 2 per SIMD):
//  * tile 256 rows x 112 weight rows x 64 K; the 112 weight rows are 7 MFMA column fragments of
//    16 = 8 gate rows + the 8 matching up rows, so silu(g) * u pairs lanes l and l ^ 8 of one
//    16-lane row (DPP row_ror:8 in the epilogue) -- no weight permutation, no [M, 2I] intermediate;
//  * waves split the rows 8 ways (32 rows each): wave tile 32 x 112 = 2 x 7 accumulators of
//    v_mfma_f32_16x16x32_bf16, every wave reads all 7 B fragments per 32-deep K step;
//  * 3-slot LDS ring (46 KiB per K-tile) filled by global_load_lds_dwordx4 (128-byte rows, chunk
//    swizzle c ^ ((row >> 1) & 7) on the source and the fragment read), two K-tiles in flight, one
//    counted vmcnt + raw s_barrier per K-tile (gemm_wide.hip's pipeline);
//  * fragment reads in inline asm with a COUNTED lgkmcnt before each MFMA that first uses a
//    fragment (hipcc otherwise waits for all 18 reads of a K-tile before its first MFMA);
//  * the next K-tile's 6 staging pieces per wave are spread over the 28 MFMAs (pinned with
//    sched_barrier); weights nontemporal (streamed once per step).
#include "common.h"
#include "launchers.h"

#include <type_traits>
#include <utility>

namespace dllm {

namespace {
constexpr int GU_BM = 256, GU_BK = 64, GU_NBUF = 3;
constexpr int GU_AEL = GU_BM * GU_BK;                       // A slot elements (bf16)
constexpr int GU_AI = 4;                                    // A pieces per wave per K-tile
constexpr int GU_RT = 2;                                    // 32-row wave band = 2 fragments

typedef __attribute__((address_space(3))) void* lds_vptr_g;
typedef __attribute__((address_space(1))) void* glb_vptr_g;

__device__ __forceinline__ int gswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void gu_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int OFF>
__device__ __forceinline__ bf16x8 gu_frag(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// s_waitcnt lgkmcnt(N) that the two fragments it names depend on (so the MFMAs using them stay
// after it); N is clamped to the counter's 15 (waiting for a few more reads than needed)
template <int N>
__device__ __forceinline__ void gu_lgkm(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "i"(N > 15 ? 15 : N));
}

// weight row of slot row r (0 .. 16 CT - 1) of column tile n_t.  SwiGLU: fragment c = r / 16,
// j = r % 16; j < 8 -> gate row, else up row, of output column n_t * 8 CT + c * 8 + (j & 7)
template <int CT, bool SWIGLU>
__device__ __forceinline__ int gu_w_row(int r, int n_t, int half) {
  if constexpr (!SWIGLU) return n_t * 16 * CT + r;
  const int c = r >> 4, j = r & 15;
  return (j >= 8 ? half : 0) + n_t * 8 * CT + c * 8 + (j & 7);
}

template <int N>
__device__ __forceinline__ void gu_lgkm1(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "i"(N > 15 ? 15 : N));
}

template <int N>
using gu_ic = std::integral_constant<int, N>;

template <int... Is, class F>
__device__ __forceinline__ void gu_for_impl(std::integer_sequence<int, Is...>, F&& f) {
  (f(gu_ic<Is>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void gu_for(F&& f) {
  gu_for_impl(std::make_integer_sequence<int, N>{}, f);
}
}  // namespace

// MODE 0: C bf16 [M, N];  1: split-K slab P (part_store, common.h) [S, M, N];  2: SwiGLU C [M, N/2].
// CT: 16-column fragments per workgroup (tile 256 x 16 CT weight rows).
template <int CT, int MODE>
__global__ void __launch_bounds__(512, 1) gemm_gu_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                         int K, int kt_per_split, int nsplit) {
  constexpr bool SWIGLU = MODE == 2;
  constexpr int BN = 16 * CT, BEL = BN * GU_BK, BUF = GU_AEL + BEL;
  constexpr int NBP = BN / 8;                                 // B pieces per K-tile
  constexpr int BI = (NBP + 7) / 8;                           // ... per wave (the excess repeat)
  constexpr int G = GU_AI + BI;                               // LDS-DMA pieces per wave per K-tile
  constexpr int NR = CT + 2;                                  // fragment reads per 32-deep K step
  constexpr int NMF = 2 * GU_RT * CT;                         // MFMAs per wave per K-tile
  constexpr int GE = NMF / (G + 1) > 0 ? NMF / (G + 1) : 1;   // a staging piece every GE MFMAs
  static_assert(GU_NBUF * BUF * 2 <= 160 * 1024, "LDS");
  static_assert(G * GE <= NMF, "pieces fit the MFMA stream");
  __shared__ __attribute__((aligned(16))) bf16 smem[GU_NBUF * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int total = gridDim.x;
  int b = blockIdx.x;
  {   // bijective XCD remap: the K slices of a column tile, then neighbouring tiles, share an XCD
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int split = b % nsplit, n_t = b / nsplit;
  const int kt0 = split * kt_per_split;
  const int nt = max(0, min(K / GU_BK, kt0 + kt_per_split) - kt0);
  const int half = N / 2;

  // staging sources: piece i covers slot rows 8 i .. 8 i + 7, lane -> (row 8 i + lane / 8, physical
  // chunk lane % 8) <- logical chunk gswz(row, lane % 8).  A: pieces 4 wv + j (rows past M clamp);
  // B: NBP pieces over 8 waves, a wave past the last repeats it (identical bytes, same LDS place)
  const bf16* srcA[GU_AI];
  const bf16* srcB[BI];
  int dstB[BI];
#pragma unroll
  for (int j = 0; j < GU_AI; ++j) {
    const int r = 8 * (wv * GU_AI + j) + (lane >> 3);
    srcA[j] = A + (size_t)min(r, M - 1) * K + (size_t)kt0 * GU_BK + gswz(r, lane & 7) * 8;
  }
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int q = min(wv * BI + j, NBP - 1);
    const int r = 8 * q + (lane >> 3);
    srcB[j] = B + (size_t)gu_w_row<CT, SWIGLU>(r, n_t, half) * K + (size_t)kt0 * GU_BK + gswz(r, lane & 7) * 8;
    dstB[j] = GU_AEL + q * 512;
  }
  // weights nontemporal when each byte is read once per step (no K split re-reads none either way)
  auto piece = [&](int buf, int t, int p) {
    bf16* base = smem + buf * BUF;
    const int ko = t * GU_BK;
    if (p < GU_AI)
      __builtin_amdgcn_global_load_lds((glb_vptr_g)(srcA[p] + ko), (lds_vptr_g)(base + (wv * GU_AI + p) * 512), 16, 0,
                                       0);
    else
      __builtin_amdgcn_global_load_lds((glb_vptr_g)(srcB[p - GU_AI] + ko), (lds_vptr_g)(base + dstB[p - GU_AI]), 16,
                                       0, 2);
  };

  // fragment read addresses: lane (row l & 15, logical chunk 4 s + l / 16) of a 16-row fragment in
  // K step s; the swizzle of row r0 + x (r0 % 16 == 0) depends on x only, so fragment f of a K step
  // sits at base_s + f * 2 KiB (immediate offsets)
  const int fr = lane & 15, fq = lane >> 4;
  const uint32_t lds0 = (uint32_t)(size_t)(lds_vptr_g)smem;
  uint32_t aoff[2], boff[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    aoff[s] = (uint32_t)(((wv * 32 + fr) * GU_BK + gswz(fr, 4 * s + fq) * 8) * 2);
    boff[s] = (uint32_t)((GU_AEL + fr * GU_BK + gswz(fr, 4 * s + fq) * 8) * 2);
  }

  f32x4 acc[GU_RT][CT];
#pragma unroll
  for (int r = 0; r < GU_RT; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one K-tile from slot `cur`; STG: stage K-tile `tn` into slot `nb` between the MFMAs.
  // Read order (2 NR reads): per K step A0 B0 .. B(CT-1) A1.  MFMA (s, rt, ct) waits for its A
  // fragment (first of its row) and its B fragment (first row) with lgkmcnt = reads issued after.
  auto ktile = [&](int cur, int nb, int tn, auto stg) {
    constexpr bool STG = decltype(stg)::value;
    const uint32_t base = lds0 + (uint32_t)(cur * BUF * 2);
    bf16x8 fa[2][GU_RT], fb[2][CT];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint32_t ab = base + aoff[s], bb = base + boff[s];
      fa[s][0] = gu_frag<0>(ab);
      gu_for<CT>([&](auto cc) { fb[s][decltype(cc)::value] = gu_frag<decltype(cc)::value * 2048>(bb); });
      fa[s][1] = gu_frag<2048>(ab);
    }
    __builtin_amdgcn_sched_barrier(0);
    gu_for<NMF>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int s = i / (GU_RT * CT), rt = (i / CT) % GU_RT, ct = i % CT;
      constexpr int need = s * NR + (rt == 0 ? 1 + ct : NR - 1);   // last read this MFMA needs
      if constexpr (rt == 0 || ct == 0) {
        gu_lgkm<2 * NR - 1 - need>(fa[s][rt], fb[s][ct]);
        __builtin_amdgcn_sched_barrier(0);
      }
      acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[s][rt], fb[s][ct], acc[rt][ct], 0, 0, 0);
      if constexpr (STG && (i % GE == GE / 2) && (i / GE < G)) piece(nb, tn, i / GE);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  if (nt > 0) {
#pragma unroll
    for (int p = 0; p < GU_NBUF - 1; ++p)
      if (p < nt)
#pragma unroll
        for (int q = 0; q < G; ++q) piece(p, p, q);
    int cur = 0, t = 0;
    for (; t + GU_NBUF - 1 < nt; ++t) {
      gu_vm<G>();                                      // K-tile t landed; t + 1 may be in flight
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int nb = cur == 0 ? GU_NBUF - 1 : cur - 1;   // slot of K-tile t - 1: free after the barrier
      ktile(cur, nb, t + GU_NBUF - 1, std::true_type{});
      cur = cur == GU_NBUF - 1 ? 0 : cur + 1;
    }
    for (; t < nt; ++t) {
      if (t + 1 < nt) gu_vm<G>(); else gu_vm<0>();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      ktile(cur, 0, 0, std::false_type{});
      cur = cur == GU_NBUF - 1 ? 0 : cur + 1;
    }
  }

  // epilogue: acc[rt][ct] lane l holds column (l & 15) of fragment ct, rows wv * 32 + rt * 16 +
  // 4 (l >> 4) + i.  SwiGLU: lane l & 15 < 8 holds the gate of output ct * 8 + (l & 7), its up
  // partner sits 8 lanes on (DPP row_ror:8 within the 16-lane row)
#pragma unroll
  for (int rt = 0; rt < GU_RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = wv * 32 + rt * 16 + 4 * fq + i;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const float v = acc[rt][ct][i];
        if constexpr (SWIGLU) {
          const float u = __int_as_float(
              __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128 /* row_ror:8 */, 0xf, 0xf, false));
          if (fr < 8 && m < M) C[(size_t)m * half + n_t * 8 * CT + ct * 8 + fr] = f2bf(silu_f(v) * u);
        } else if (m < M) {
          const int n = n_t * BN + ct * 16 + fr;
          if constexpr (MODE == 1) part_store(P, ((size_t)split * M + m) * N + n, v);
          else C[(size_t)m * N + n] = f2bf(v);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------
// AREG form: the activations bypass LDS.  With 32-row bands each wave's A fragments are its own
// (no other wave reads them), so they are loaded straight into VGPRs in MFMA operand layout
// (16 contiguous bytes per lane: row l & 15, K 8 (l >> 4) .. + 8) three K-tiles ahead; only the
// weight tile goes through the LDS ring (16 CT rows x 128 B per slot, NB slots).  Per K-tile and
// CU this drops the LDS traffic from 32 KiB A staging + 8 x 2 KiB A fragment reads + the B share
// to the B share alone (the LDS array sat ~85 % busy feeding the MFMAs in the form above).
// Issue order per K-tile j (counted vmcnt): B pieces of K-tile j + NB - 1 between the MFMAs, then
// the 4 A loads of K-tile j + 3 at its end (into the ring registers K-tile j just released).
// ---------------------------------------------------------------------------------------------
// The A loads are inline asm so that hipcc's waitcnt pass leaves the counting to the kernel (with
// plain loads it drains vmcnt(0) at every loop head).  The asm destination looks written at issue,
// so: early-clobber (never shares a register with the address), every ring register stays live
// until a wait that names it (`+v`), and the kernel's last wait names all of them (the tail's
// clamped loads must land before the epilogue may reuse their registers).
__device__ __forceinline__ bf16x8 gua_load(const bf16* p) {
  bf16x8 r;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=&v"(r) : "v"(p) : "memory");
  return r;
}

template <int CT, int MODE, int NB>
__global__ void __launch_bounds__(512, 1) gemm_gua_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                          int K, int kt_per_split, int nsplit) {
  constexpr bool SWIGLU = MODE == 2;
  constexpr int BN = 16 * CT, BUF = BN * GU_BK;              // LDS slot: the weight tile only
  constexpr int NBP = BN / 8, BI = (NBP + 7) / 8;            // B pieces per K-tile / per wave
  constexpr int DA = 3;                                       // A K-tiles held in registers
  constexpr int NMF = 2 * GU_RT * CT;
  constexpr int GE = NMF / (BI + 1) > 0 ? NMF / (BI + 1) : 1;
  constexpr int VWAIT = (DA - 1) * (BI + 4);                  // ops younger than K-tile t's A loads
  static_assert(NB >= 4 && NB * BUF * 2 <= 160 * 1024, "ring");
  static_assert(VWAIT <= 63, "vmcnt");
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * BUF];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int total = gridDim.x;
  int b = blockIdx.x;
  {
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int split = b % nsplit, n_t = b / nsplit;
  const int kt0 = split * kt_per_split;
  const int nt = max(0, min(K / GU_BK, kt0 + kt_per_split) - kt0);
  const int half = N / 2;
  const int fr = lane & 15, fq = lane >> 4;

  // A: this lane's operand rows (clamped past M) and K offset within a 32-deep step
  const bf16* arow[GU_RT];
#pragma unroll
  for (int rt = 0; rt < GU_RT; ++rt)
    arow[rt] = A + (size_t)min(wv * 32 + rt * 16 + fr, M - 1) * K + (size_t)kt0 * GU_BK + fq * 8;
  // B staging (as gemm_gu_kernel)
  const bf16* srcB[BI];
  int dstB[BI];
#pragma unroll
  for (int j = 0; j < BI; ++j) {
    const int q = min(wv * BI + j, NBP - 1);
    const int r = 8 * q + (lane >> 3);
    srcB[j] = B + (size_t)gu_w_row<CT, SWIGLU>(r, n_t, half) * K + (size_t)kt0 * GU_BK + gswz(r, lane & 7) * 8;
    dstB[j] = q * 512;
  }
  // K-tiles past this split's range (the pipeline's tail) re-load the last one: static op counts
  auto bpiece = [&](int slot, int t, int j) {
    t = min(t, nt - 1);
    __builtin_amdgcn_global_load_lds((glb_vptr_g)(srcB[j] + t * GU_BK), (lds_vptr_g)(smem + slot * BUF + dstB[j]), 16,
                                     0, 2);
  };
  bf16x8 fa[DA][2][GU_RT];                                  // [ring][K step][row fragment]
  auto aload = [&](bf16x8 (&dst)[2][GU_RT], int t) {
    t = min(t, nt - 1);
#pragma unroll
    for (int st = 0; st < 2; ++st)
#pragma unroll
      for (int rt = 0; rt < GU_RT; ++rt) dst[st][rt] = gua_load(arow[rt] + t * GU_BK + st * 32);
  };

  const uint32_t lds0 = (uint32_t)(size_t)(lds_vptr_g)smem;
  uint32_t boff[2];
#pragma unroll
  for (int st = 0; st < 2; ++st) boff[st] = (uint32_t)((fr * GU_BK + gswz(fr, 4 * st + fq) * 8) * 2);

  f32x4 acc[GU_RT][CT];
#pragma unroll
  for (int r = 0; r < GU_RT; ++r)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  // K-tile t (slot t % NB, A ring slot R): wait for its A registers and B slot, barrier, B
  // fragment reads (counted lgkmcnt per first use), MFMAs with the B pieces of K-tile t + NB - 1
  // spread between them, then the A loads of K-tile t + DA into ring slot R
  // W: ops issued after K-tile t's A loads (VWAIT in the steady state, fewer in the first DA - 1
  // K-tiles, whose A loads sit in the prologue)
  auto step = [&](int t, auto rc, auto wc) {
    constexpr int R = decltype(rc)::value, W = decltype(wc)::value;
    asm volatile("s_waitcnt vmcnt(%4)" : "+v"(fa[R][0][0]), "+v"(fa[R][0][1]), "+v"(fa[R][1][0]), "+v"(fa[R][1][1])
                 : "i"(W) : "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int cur = t % NB, nb = (t + NB - 1) % NB;
    const uint32_t base = lds0 + (uint32_t)(cur * BUF * 2);
    bf16x8 fb[2][CT];
#pragma unroll
    for (int st = 0; st < 2; ++st)
      gu_for<CT>([&](auto cc) { fb[st][decltype(cc)::value] = gu_frag<decltype(cc)::value * 2048>(base + boff[st]); });
    __builtin_amdgcn_sched_barrier(0);
    gu_for<NMF>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int st = i / (GU_RT * CT), rt = (i / CT) % GU_RT, ct = i % CT;
      if constexpr (rt == 0) {
        gu_lgkm1<2 * CT - 1 - (st * CT + ct)>(fb[st][ct]);
        __builtin_amdgcn_sched_barrier(0);
      }
      acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[R][st][rt], fb[st][ct], acc[rt][ct], 0, 0, 0);
      if constexpr ((i % GE == GE / 2) && (i / GE < BI)) bpiece(nb, t + NB - 1, i / GE);
      __builtin_amdgcn_sched_barrier(0);
    });
    aload(fa[R], t + DA);
    __builtin_amdgcn_sched_barrier(0);
  };

  if (nt > 0) {
    // prologue: B K-tiles 0 .. NB - 2 into their slots (one issue group per K-tile, in the order
    // the loop's counts assume: the B group of K-tile j precedes the A group of K-tile j + DA ...)
    // -- simplest static order: every B group, then the A groups of K-tiles 0 .. DA - 1
#pragma unroll
    for (int j = 0; j < NB - 1; ++j)
#pragma unroll
      for (int q = 0; q < BI; ++q) bpiece(j, j, q);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < DA; ++j) {
      aload(fa[j], j);
      __builtin_amdgcn_sched_barrier(0);
    }
    static_assert(DA == 3, "the loop below is unrolled for DA = 3");
    // K-tile t < DA: younger than its A group are the later prologue A groups and t full K-tiles
    // (the host guarantees nt >= DA per split: no branch here, so hipcc's own vmcnt scoreboard
    // reaches the loop with one pending-op pattern and keeps counted waits)
    step(0, gu_ic<0>{}, gu_ic<4 * (DA - 1)>{});
    step(1, gu_ic<1>{}, gu_ic<4 * (DA - 2) + (BI + 4)>{});
    step(2, gu_ic<2>{}, gu_ic<VWAIT>{});
    int t = DA;
    for (; t + DA <= nt; t += DA) {
      step(t, gu_ic<0>{}, gu_ic<VWAIT>{});
      step(t + 1, gu_ic<1>{}, gu_ic<VWAIT>{});
      step(t + 2, gu_ic<2>{}, gu_ic<VWAIT>{});
    }
    if (t < nt) step(t, gu_ic<0>{}, gu_ic<VWAIT>{});
    if (t + 1 < nt) step(t + 1, gu_ic<1>{}, gu_ic<VWAIT>{});
  }
  static_assert(DA == 3 && GU_RT == 2, "final wait names every ring register");
  asm volatile("s_waitcnt vmcnt(0)"
               : "+v"(fa[0][0][0]), "+v"(fa[0][0][1]), "+v"(fa[0][1][0]), "+v"(fa[0][1][1]), "+v"(fa[1][0][0]),
                 "+v"(fa[1][0][1]), "+v"(fa[1][1][0]), "+v"(fa[1][1][1]), "+v"(fa[2][0][0]), "+v"(fa[2][0][1]),
                 "+v"(fa[2][1][0]), "+v"(fa[2][1][1])
               :
               : "memory");

#pragma unroll
  for (int rt = 0; rt < GU_RT; ++rt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = wv * 32 + rt * 16 + 4 * fq + i;
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const float v = acc[rt][ct][i];
        if constexpr (SWIGLU) {
          const float u = __int_as_float(
              __builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128 /* row_ror:8 */, 0xf, 0xf, false));
          if (fr < 8 && m < M) C[(size_t)m * half + n_t * 8 * CT + ct * 8 + fr] = f2bf(silu_f(v) * u);
        } else if (m < M) {
          const int n = n_t * BN + ct * 16 + fr;
          if constexpr (MODE == 1) part_store(P, ((size_t)split * M + m) * N + n, v);
          else C[(size_t)m * N + n] = f2bf(v);
        }
      }
    }
}

// C [M, I] = silu(A Wg^T) * (A Wu^T), W = [Wg; Wu] [2I, K]; 1 <= M <= 256, I % 56 == 0, K % 64 == 0.
void gemm_gate_up(uintptr_t c, uintptr_t a, uintptr_t w, int M, int I, int K, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1 && M <= GU_BM, "gemm_gate_up: 1 <= M <= 256");
  DLLM_HOST_CHECK(I % 56 == 0, "gemm_gate_up: I must be a multiple of 56");
  DLLM_HOST_CHECK(K % GU_BK == 0 && K >= GU_BK, "gemm_gate_up: K must be a positive multiple of 64");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // variant 1: activations straight into registers (gemm_gua_kernel), 6-slot weight ring
  if (variant == 1) {
    DLLM_HOST_CHECK(K >= 3 * GU_BK, "gemm_gate_up variant 1: K >= 192");
    hipLaunchKernelGGL((gemm_gua_kernel<7, 2, 6>), dim3(I / 56), dim3(512), 0, s, (const bf16*)a, (const bf16*)w,
                       (bf16*)c, (float*)nullptr, M, 2 * I, K, K / GU_BK, 1);
  } else
    hipLaunchKernelGGL((gemm_gu_kernel<7, 2>), dim3(I / 56), dim3(512), 0, s, (const bf16*)a, (const bf16*)w, (bf16*)c,
                       (float*)nullptr, M, 2 * I, K, K / GU_BK, 1);
  DLLM_HIP_CHECK(hipGetLastError());
}

// Plain / split-K form: C = A B^T (mode 0) or split-K slabs in ws (mode 2, S > 1, natural column
// order as gemm_wide's); 1 <= M <= 256; N % (16 CT) == 0 with CT = ct (6, 7 or 8).  Returns S.
int gemm_band(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
              int mode, int ct, uintptr_t stream) {
  const bool areg = (ct & 256) != 0;                         // ct | 256: gemm_gua_kernel (A in registers)
  ct &= 255;
  DLLM_HOST_CHECK(M >= 1 && M <= GU_BM, "gemm_band: 1 <= M <= 256");
  DLLM_HOST_CHECK(ct == 6 || ct == 7 || ct == 8, "gemm_band: ct in 6, 7, 8");
  DLLM_HOST_CHECK(N % (16 * ct) == 0, "gemm_band: N % (16 ct)");
  DLLM_HOST_CHECK(K % GU_BK == 0 && K >= GU_BK, "gemm_band: K must be a positive multiple of 64");
  DLLM_HOST_CHECK(mode == 0 || mode == 2, "gemm_band: mode 0 (bf16) or 2 (slabs)");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  const int ktiles = K / GU_BK, kts = (ktiles + splits - 1) / splits, S = (ktiles + kts - 1) / kts;
  // gemm_gua_kernel runs >= 3 K-tiles in every split (its pipeline prologue is unconditional)
  DLLM_HOST_CHECK(!areg || (kts >= 3 && ktiles - (S - 1) * kts >= 3), "gemm_band areg: >= 3 K-tiles per split");
  DLLM_HOST_CHECK(mode == 0 ? S == 1 : S > 1, "gemm_band: mode 2 needs a K split, mode 0 none");
  if (S > 1) DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const unsigned grid = (unsigned)((N / (16 * ct)) * S);
#define DLLM_BAND_GO(CT_, MODE_)                                                                                 \
  do {                                                                                                          \
    if (areg)                                                                                                   \
      hipLaunchKernelGGL((gemm_gua_kernel<CT_, MODE_, 6>), dim3(grid), dim3(512), 0, s, (const bf16*)a,          \
                         (const bf16*)b, (bf16*)c, (float*)ws, M, N, K, kts, S);                                 \
    else                                                                                                        \
      hipLaunchKernelGGL((gemm_gu_kernel<CT_, MODE_>), dim3(grid), dim3(512), 0, s, (const bf16*)a, (const bf16*)b, \
                         (bf16*)c, (float*)ws, M, N, K, kts, S);                                                 \
  } while (0)
  if (S == 1) {
    if (ct == 6) DLLM_BAND_GO(6, 0); else if (ct == 7) DLLM_BAND_GO(7, 0); else DLLM_BAND_GO(8, 0);
  } else {
    if (ct == 6) DLLM_BAND_GO(6, 1); else if (ct == 7) DLLM_BAND_GO(7, 1); else DLLM_BAND_GO(8, 1);
  }
#undef DLLM_BAND_GO
  DLLM_HIP_CHECK(hipGetLastError());
  return S;
}

}  // namespace dllm
