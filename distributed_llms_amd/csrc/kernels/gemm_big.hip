// Decode GEMM experiment for M = 256 with ONE wave per SIMD: C[M,N] = A[M,K] . B[N,K]^T, bf16 in,
// f32 accumulate, a 256 x 256 tile per workgroup of 4 waves (2 (M) x 2 (N)), wave tile 128 x 128.
//
// Why: the wide kernel's (gemm_wide.hip, 256 x 128 tile, 8 waves of 64 x 64) K loop is mostly its
// MFMA / LDS-read phase (no staging loads: 52 of 66 us on the MLP up projection, MFMA ~50 % busy):
// every 16x16x32 MFMA of a 64 x 64 wave tile needs half a fragment read, which with two waves per
// SIMD leaves the matrix pipe waiting.  A 128 x 128 wave tile needs a quarter fragment per MFMA
// and the 64 independent accumulators of one wave keep the pipe fed; one wave per SIMD gets the
// whole 512-register file (256 accumulator registers).  The tile also halves the activation bytes
// each workgroup re-stages per FLOP.  gemm_sq.hip tried the 256 x 256 tile with 8 waves, two 64 KiB
// buffers and one tile in flight; here K-tiles are 32 deep (32 KiB) so four buffers keep three
// tiles in flight.
//
// Structure (gfx950, wave64, 256 threads):
//  * K-tile of 32: every LDS row is 64 B = 4 16-byte chunks; an MFMA operand fragment is one chunk
//    (lane: row lane & 15, chunk lane >> 4), one ds_read_b128.  Bank swizzle: chunk c of row r sits
//    in slot c ^ ((r >> 2) & 2) -- for each of ds_read_b128's four 16-lane groups the 16 (row,
//    slot) pairs then cover the 16 bank quads once (derivation in profiles/wide_gemm.md);
//  * global -> LDS by global_load_lds_dwordx4 (16 rows x 64 B per wave-instruction; the swizzle on
//    the per-lane SOURCE address), 8 per wave per K-tile, spread between the tile's 64 MFMAs;
//  * four LDS buffers, counted vmcnt + one raw s_barrier per K-tile (never vmcnt(0) in the loop);
//  * XCD-aware bijective block remap (the K slices of one N tile run back-to-back on one XCD);
//  * split-K only, slabs in natural column order (common.h part_store): the MLP gate|up's SwiGLU
//    is applied by splitk_reduce(_swiglu), the other projections defer into the next norm.
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace dllm {

namespace {
constexpr int GBM = 256, GBN = 256, GBK = 32, GNB = 4;
constexpr int GAEL = GBM * GBK, GBEL = GBN * GBK, GBUF = GAEL + GBEL;   // bf16 elements (32 KiB)
constexpr int GPIECES = (GBM + GBN) / 16 / 4;                            // glds per wave per K-tile (8)
typedef __attribute__((address_space(3))) void* lds_vptr_g;
typedef __attribute__((address_space(1))) void* glb_vptr_g;

__device__ __forceinline__ int gslot(int row, int chunk) { return chunk ^ ((row >> 2) & 2); }

#define DLLM_GVM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
__device__ __forceinline__ void gwait(int younger) {    // younger staged tiles allowed in flight
  if (younger >= 2) DLLM_GVM(16);
  else if (younger == 1) DLLM_GVM(8);
  else DLLM_GVM(0);
}
#undef DLLM_GVM
}  // namespace

template <bool SPLIT>
__global__ void __launch_bounds__(256, 1) gemm_big_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                          bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                          int K, int kt_per_split, int nsplit) {
  __shared__ __attribute__((aligned(16))) bf16 smem[GNB * GBUF];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  const int mtiles = (M + GBM - 1) / GBM;
  const int total = gridDim.x;
  int b = blockIdx.x;
  {
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  const int m_t = b % mtiles, rest = b / mtiles;
  const int split = rest % nsplit, n_t = rest / nsplit;
  const int m0 = m_t * GBM;
  const int kt0 = split * kt_per_split;
  const int nt = max(0, min(K / GBK, kt0 + kt_per_split) - kt0);

  // staging: wave-instruction i = wv * 8 + j covers operand rows 16 (i % 16) .. +15 (A for i < 16,
  // B otherwise); lane -> row 16 (i % 16) + lane / 4, LDS slot lane % 4 <- source chunk slot ^ swz
  uint32_t off[GPIECES];
#pragma unroll
  for (int j = 0; j < GPIECES; ++j) {
    const int i = wv * GPIECES + j;
    const int r = 16 * (i & 15) + (lane >> 2);
    const int c = gslot(r, lane & 3);
    off[j] = i < 16 ? (uint32_t)(min(m0 + r, M - 1) * K + kt0 * GBK + c * 8)
                    : (uint32_t)((n_t * GBN + r) * K + kt0 * GBK + c * 8);
  }
  auto piece = [&](bf16* base, int ko, int j) {
    const int i = wv * GPIECES + j;
    const bf16* src = (i < 16 ? A : B) + off[j] + ko;
    __builtin_amdgcn_global_load_lds((glb_vptr_g)src, (lds_vptr_g)(base + (i < 16 ? 0 : GAEL) + (i & 15) * 512), 16,
                                     0, 0);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  // per-lane LDS element offsets of this wave's fragments (row rt * 16 + fr of its 128-row band)
  const int arow = wm * 128 + fr, brow = wn * 128 + fr;
  const int aoff = arow * GBK + gslot(arow, fq) * 8;          // + rt * 16 * GBK (slot unchanged)
  const int boff = GAEL + brow * GBK + gslot(brow, fq) * 8;

  auto ktile = [&](int cur, bf16* dst, int ko, auto stg) {
    constexpr bool STG = decltype(stg)::value;
    const bf16* base = smem + cur * GBUF;
    bf16x8 fa[8], fb[8];
#pragma unroll
    for (int rt = 0; rt < 8; ++rt) fa[rt] = *reinterpret_cast<const bf16x8*>(base + aoff + rt * 16 * GBK);
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) fb[ct] = *reinterpret_cast<const bf16x8*>(base + boff + ct * 16 * GBK);
#pragma unroll
    for (int rt = 0; rt < 8; ++rt)
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt], fb[ct], acc[rt][ct], 0, 0, 0);
        if constexpr (STG) {
          const int n = rt * 8 + ct;                       // one staging piece every 8 MFMAs
          if ((n & 7) == 3) piece(dst, ko, n >> 3);
        }
      }
  };

  if (nt > 0) {
#pragma unroll
    for (int p = 0; p < GNB - 1; ++p)
      if (p < nt) {
#pragma unroll
        for (int j = 0; j < GPIECES; ++j) piece(smem + p * GBUF, p * GBK, j);
      }
    int cur = 0, t = 0;
    for (; t + GNB - 1 < nt; ++t) {
      gwait(GNB - 2);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      const int nb = cur == 0 ? GNB - 1 : cur - 1;         // read in iteration t - 1, before the barrier
      ktile(cur, smem + nb * GBUF, (t + GNB - 1) * GBK, std::true_type{});
      cur = cur == GNB - 1 ? 0 : cur + 1;
    }
    for (; t < nt; ++t) {
      gwait(nt - 1 - t);
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      ktile(cur, smem, 0, std::false_type{});
      cur = cur == GNB - 1 ? 0 : cur + 1;
    }
  }

  // epilogue: acc[rt][ct] lane holds tile column fr of fragment ct, rows 4 fq + i of fragment rt
#pragma unroll
  for (int rt = 0; rt < 8; ++rt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 128 + rt * 16 + 4 * fq + i;
      if (m >= M) continue;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const int n = n_t * GBN + wn * 128 + ct * 16 + fr;
        if (SPLIT) part_store(P, ((size_t)split * M + m) * N + n, acc[rt][ct][i]);
        else C[(size_t)m * N + n] = f2bf(acc[rt][ct][i]);
      }
    }
  }
}

// mode 0: C = A B^T;  mode 1: SwiGLU over B = [Bg; Bu] (split-K required: applied by the reduce);
// mode 2: leave the split-K partial slabs in ws (S > 1).  Returns the K slice count S.
int gemm_big(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
             int mode, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1 && M <= 4 * GBM, "1 <= M <= 1024");
  DLLM_HOST_CHECK(K % GBK == 0, "K must be a multiple of 32");
  DLLM_HOST_CHECK(N % GBN == 0, "N must be a multiple of 256");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ktiles = K / GBK;
  const int kts = (ktiles + splits - 1) / splits;
  const int S = (ktiles + kts - 1) / kts;
  DLLM_HOST_CHECK(mode == 0 || S > 1, "SwiGLU / deferred modes need a K split");
  const int mtiles = (M + GBM - 1) / GBM;
  const long grid = (long)(N / GBN) * mtiles * S;
  DLLM_HOST_CHECK(grid >= 1 && grid < (1L << 31), "grid");
  DLLM_HOST_CHECK((long)M * K < (1L << 32) && (long)N * K < (1L << 32), "32-bit staging offsets");
  if (S == 1) {
    hipLaunchKernelGGL((gemm_big_kernel<false>), dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)a,
                       (const bf16*)b, (bf16*)c, (float*)ws, M, N, K, kts, S);
    DLLM_HIP_CHECK(hipGetLastError());
    return 1;
  }
  DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  hipLaunchKernelGGL((gemm_big_kernel<true>), dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)a, (const bf16*)b,
                     (bf16*)c, (float*)ws, M, N, K, kts, S);
  DLLM_HIP_CHECK(hipGetLastError());
  if (mode == 2) return S;
  splitk_reduce_ex(c, ws, 0, S, M, N, mode == 1 ? 1 : 0, stream);
  return S;
}

}  // namespace dllm
