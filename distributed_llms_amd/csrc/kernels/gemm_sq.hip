// Decode GEMM for 128 < M <= 256 with a 256 x 256 tile: C[M,N] = A[M,K] . B[N,K]^T, bf16 in, f32
// accumulate.  Sibling of gemm_wide.hip (256 x 128 tiles), in its own translation unit so the two
// kernels' register allocation does not perturb each other (guide §5.4 rule 19).
//
// Why a wider N tile: at M = 256 the wide kernel's workgroups are bound by what one CU can pull
// through L2 -> LDS (profiles/wide_gemm.md: ~45 GB/s per CU; removing the staging loads makes the
// loop 21 % faster), and two thirds of those bytes are the activation tile A, which every N tile
// re-reads.  Per K-tile a 256 x 256 tile stages 64 KiB for 2x the MFMA work of a 256 x 128 tile
// (48 KiB): bytes per FLOP drop by a third, and with 12 fragment reads per 32 MFMAs (8 A + 4 B per
// wave, wave tile 128 x 64) instead of 16, so does the LDS read traffic.  The price: only two
// 64 KiB LDS buffers fit (one tile in flight while the other is multiplied), and half as many
// N tiles, so the projections need deeper K splits to fill 256 CUs (qkv 10, o / down 16, MLP
// gate|up 2 -- the SwiGLU is then applied by the split-K reduce).
//
// Structure (gfx950, wave64, 512 threads = 8 waves as 2 (M) x 4 (N), 8 x 4 accumulators of
// v_mfma_f32_16x16x32_bf16 per wave):
//  * global -> LDS by global_load_lds_dwordx4, 8 rows x 128 B per wave-instruction, bank swizzle
//    chunk ^ ((row >> 1) & 7) on the per-lane SOURCE address and on the ds_read address (rule 21);
//  * tile t + 1's eight LDS-DMA pieces per thread are issued between tile t's MFMAs; one
//    vmcnt(0) + raw s_barrier per K-tile; all LDS in one __shared__ array (trap 4a);
//  * XCD-aware bijective block remap (the K slices of one N tile run back-to-back on one XCD);
//  * SwiGLU without a split: 16-row groups alternate gate / up rows so that a lane holds gate and up
//    of one output column in neighbouring accumulators (as in gemm_wide.hip);
//  * split-K: f16 x 2^-6 partial slabs in natural column order (common.h), reduced by
//    splitk_reduce(_swiglu) or deferred into splitk_add_rms_norm.
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace dllm {

namespace {
constexpr int QBM = 256, QBN = 256, QBK = 64;
constexpr int QAEL = QBM * QBK, QBEL = QBN * QBK, QBUF = QAEL + QBEL;   // bf16 elements (64 KiB)
constexpr int QAI = 4, QBI = 4, QG = QAI + QBI;                         // glds per thread per tile
constexpr int QRT = 8, QCT = 4;                                         // 16 x 16 fragments per wave

typedef __attribute__((address_space(3))) void* lds_vptr_q;
typedef __attribute__((address_space(1))) void* glb_vptr_q;

__device__ __forceinline__ int qswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// B-tile row r (0..255) -> weight row.  SwiGLU: 16-row group g alternates gate (even g) and up
// (odd g) rows of output columns n_t * 128 + (g / 2) * 16 + r % 16.
template <bool SWIGLU>
__device__ __forceinline__ int sq_b_row(int r, int n_t, int half) {
  if (!SWIGLU) return n_t * QBN + r;
  const int g = r >> 4;
  return ((g & 1) ? half : 0) + n_t * 128 + (g >> 1) * 16 + (r & 15);
}
}  // namespace

// VAR bit 0..1: weight cache policy (2 = nontemporal); bit 2 (EARLY): issue all of tile t + 1's
// staging pieces right after the barrier instead of spreading them over tile t's MFMAs
template <bool SPLIT, bool SWIGLU, int VAR>
__global__ void __launch_bounds__(512, 1) gemm_sq_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                         int K, int kt_per_split, int nsplit) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * QBUF];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 2, wn = wv & 3;
  const int mtiles = (M + QBM - 1) / QBM;
  const int total = gridDim.x;
  int b = blockIdx.x;
  {
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int m_t = b % mtiles, rest = b / mtiles;
  const int split = rest % nsplit, n_t = rest / nsplit;
  const int m0 = m_t * QBM;
  const int kt0 = split * kt_per_split;
  const int nt = max(0, min(K / QBK, kt0 + kt_per_split) - kt0);

  // per-lane staging sources for K-tile 0 as 32-bit element offsets (every operand here has
  // < 2^31 elements; 64-bit pointers would cost 8 more VGPRs in a kernel at the 256 cap):
  // instruction i = wv * 4 + j covers tile rows 8i .. 8i+7
  uint32_t offA[QAI], offB[QBI];
#pragma unroll
  for (int j = 0; j < QAI; ++j) {
    const int r = 8 * (wv * QAI + j) + (lane >> 3);
    offA[j] = (uint32_t)(min(m0 + r, M - 1) * K + kt0 * QBK + qswz(r, lane & 7) * 8);
  }
#pragma unroll
  for (int j = 0; j < QBI; ++j) {
    const int r = 8 * (wv * QBI + j) + (lane >> 3);
    offB[j] = (uint32_t)(sq_b_row<SWIGLU>(r, n_t, N / 2) * K + kt0 * QBK + qswz(r, lane & 7) * 8);
  }
  // weights streamed nontemporally (read once) where the grid has no K split (VAR 2)
  constexpr int BAUX = (VAR & 3) == 2 ? 2 : 0;
  constexpr bool EARLY = (VAR & 4) != 0;
  constexpr bool NOSTAGE = (VAR & 8) != 0;      // ablation (wrong results): no staging in the loop
  constexpr bool NOPIN = (VAR & 16) != 0;       // ablation: no sched_barrier between substeps
  auto piece = [&](bf16* base, int ko, int p) {
    if (p < QAI)
      __builtin_amdgcn_global_load_lds((glb_vptr_q)(A + offA[p] + ko), (lds_vptr_q)(base + (wv * QAI + p) * 512), 16,
                                       0, 0);
    else
      __builtin_amdgcn_global_load_lds((glb_vptr_q)(B + offB[p - QAI] + ko),
                                       (lds_vptr_q)(base + QAEL + (wv * QBI + p - QAI) * 512), 16, 0, BAUX);
  };

  f32x4 acc[QRT][QCT];
#pragma unroll
  for (int a = 0; a < QRT; ++a)
#pragma unroll
    for (int c = 0; c < QCT; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // one K-tile of MFMAs from buffer `cur`; with STG the next tile's QG pieces go out in between
  auto ktile = [&](int cur, bf16* dst, int ko, auto stg) {
    constexpr bool STG = decltype(stg)::value;
    const bf16* sa = smem + cur * QBUF;
    const bf16* sb = sa + QAEL;
    constexpr int NMF = 2 * QRT * QCT;        // 64 MFMAs per wave per K-tile
    constexpr int EVERY = NMF / (QG + 1);     // one staging piece every 7 MFMAs
    if constexpr (STG && EARLY && !NOSTAGE) {
#pragma unroll
      for (int p = 0; p < QG; ++p) piece(dst, ko, p);
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 fa[QRT], fb[QCT];
#pragma unroll
      for (int rt = 0; rt < QRT; ++rt) {
        const int row = wm * 128 + rt * 16 + fr;
        fa[rt] = *reinterpret_cast<const bf16x8*>(sa + row * QBK + qswz(row, 4 * s + fq) * 8);
      }
#pragma unroll
      for (int ct = 0; ct < QCT; ++ct) {
        const int row = wn * 64 + ct * 16 + fr;
        fb[ct] = *reinterpret_cast<const bf16x8*>(sb + row * QBK + qswz(row, 4 * s + fq) * 8);
      }
#pragma unroll
      for (int rt = 0; rt < QRT; ++rt)
#pragma unroll
        for (int ct = 0; ct < QCT; ++ct) {
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt], fb[ct], acc[rt][ct], 0, 0, 0);
          if constexpr (STG && !EARLY && !NOSTAGE) {
            const int i = (s * QRT + rt) * QCT + ct + 1;
            if (i % EVERY == 0 && i / EVERY <= QG) piece(dst, ko, i / EVERY - 1);
          }
        }
      // keep the next substep's 12 fragment reads below this one's MFMAs: hoisting them would
      // need 48 more VGPRs than the 256 a 2-wave-per-SIMD workgroup has (128 go to accumulators);
      // the partner wave on the SIMD covers their latency
      if constexpr (!NOPIN) __builtin_amdgcn_sched_barrier(0);
    }
  };

  if (nt > 0) {
#pragma unroll
    for (int p = 0; p < QG; ++p) piece(smem, 0, p);
    // steady state: tile t has landed (this wave's pieces: vmcnt(0); every wave's: the barrier),
    // and buffer (t + 1) % 2 is free -- tile t - 1's fragments were consumed by MFMAs issued
    // before the barrier -- so tile t + 1 is staged into it while tile t is multiplied.  The last
    // tile is peeled off (no staging): one loop body, no per-iteration branch between two copies
    // of the MFMA block (that merge cost ~100 spilled VGPRs)
    int cur = 0;
    for (int t = 0; t + 1 < nt; ++t) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      ktile(cur, smem + (cur ^ 1) * QBUF, (t + 1) * QBK, std::true_type{});
      cur ^= 1;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    ktile(cur, smem, 0, std::false_type{});
  }

  // epilogue: acc[rt][ct] lane holds tile column (lane & 15), rows 4 * (lane >> 4) + i
#pragma unroll
  for (int rt = 0; rt < QRT; ++rt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 128 + rt * 16 + 4 * fq + i;
      if (m >= M) continue;
      if (SWIGLU && !SPLIT) {
        const int half = N / 2;
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int c = n_t * 128 + (wn * 2 + p) * 16 + fr;
          C[(size_t)m * half + c] = f2bf(silu_f(acc[rt][2 * p][i]) * acc[rt][2 * p + 1][i]);
        }
      } else {
#pragma unroll
        for (int ct = 0; ct < QCT; ++ct) {
          const int n = sq_b_row<SWIGLU>(wn * 64 + ct * 16 + fr, n_t, N / 2);
          if (SPLIT) part_store(P, ((size_t)split * M + m) * N + n, acc[rt][ct][i]);
          else C[(size_t)m * N + n] = f2bf(acc[rt][ct][i]);
        }
      }
    }
  }
}

// mode 0: C = A B^T;  mode 1: SwiGLU, C[M, N/2] = silu(A Bg^T) * (A Bu^T) with B = [Bg; Bu];
// mode 2: leave the split-K partial slabs in ws (S > 1 required).  Returns the K slice count S.
int gemm_sq(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
            int mode, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1 && M <= 4 * QBM, "1 <= M <= 1024");
  DLLM_HOST_CHECK(K % QBK == 0, "K must be a multiple of 64");
  DLLM_HOST_CHECK(N % QBN == 0, "N must be a multiple of 256");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ktiles = K / QBK;
  const int kts = (ktiles + splits - 1) / splits;
  const int S = (ktiles + kts - 1) / kts;
  DLLM_HOST_CHECK(mode != 2 || S > 1, "mode 2 needs a K split");
  const int mtiles = (M + QBM - 1) / QBM;
  const long grid = (long)(N / QBN) * mtiles * S;
  DLLM_HOST_CHECK(grid >= 1 && grid < (1L << 31), "grid");
#define DLLM_SQ_GO(SPLIT_, SW_, V_)                                                                        \
  hipLaunchKernelGGL((gemm_sq_kernel<SPLIT_, SW_, V_>), dim3((unsigned)grid), dim3(512), 0, s, (const bf16*)a, \
                     (const bf16*)b, (bf16*)c, (float*)ws, M, N, K, kts, S)
  const bool early = variant & 4;
  if (S == 1) {
    if (mode == 1) { if (early) DLLM_SQ_GO(false, true, 6); else DLLM_SQ_GO(false, true, 2); }
    else { if (early) DLLM_SQ_GO(false, false, 6); else DLLM_SQ_GO(false, false, 2); }
    DLLM_HIP_CHECK(hipGetLastError());
    return 1;
  }
  DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  // split: natural column order (the SwiGLU, if any, is applied by the reduce)
  if (variant == 12) DLLM_SQ_GO(true, false, 13);        // ablations (A/B only)
  else if (variant == 20) DLLM_SQ_GO(true, false, 21);
  else if (early) DLLM_SQ_GO(true, false, 5);
  else DLLM_SQ_GO(true, false, 1);
#undef DLLM_SQ_GO
  DLLM_HIP_CHECK(hipGetLastError());
  if (mode == 2) return S;
  splitk_reduce_ex(c, ws, 0, S, M, N, mode == 1 ? 1 : 0, stream);
  return S;
}

}  // namespace dllm
