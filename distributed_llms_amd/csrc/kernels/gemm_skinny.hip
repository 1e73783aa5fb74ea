// K3/K8/K9/K10: decode-shaped GEMM, Y[M,N] = X[M,K] . W[N,K]^T, M <= 64, bf16 in/out.
//
// Regime: weight streaming.  At decode batch sizes every weight byte is used M times, so
// the kernel has to pull W from HBM near the ~6 TB/s ceiling.
//
// Structure (gfx950, wave64, v_mfma_f32_16x16x32_bf16):
//  * one workgroup = 8 waves = one tile of NT x 16 output columns and ALL M rows; the 8
//    waves split K (contiguous ranges), so there is no cross-workgroup reduction: a split-K
//    seam with an agent-scope release/acquire hand-off costs more than it saves at these
//    sizes (measured: fences per workgroup dominated the first version of this kernel,
//    profiles/gemm_skinny_v1.txt; guide price list rows splitk-seam / publish-large);
//  * W and X fragments go straight to VGPRs (operand streamed once, guide "GEMV/M<=16" row);
//    W with non-temporal loads (read once per step, never re-read from L2/MALL);
//  * k is permuted inside each 128-wide k-group identically for X and W (skinny_common.h):
//    load i of lane (r, g) reads elements 32i + 8g..+7 of row r, so one wave-instruction
//    covers 64 contiguous bytes of each of 16 rows.  The first layout (8i + 32g) touched 32
//    lines per instruction and only tied hipBLASLt; this one streams 4-5 TB/s at M <= 4
//    (profiles/gemm_skinny_v3_vs_hipblaslt.txt);
//  * waves combine their partial tiles with LDS float atomics (ds_add_f32) into one
//    [M_pad x BN] f32 tile; the epilogue writes bf16 (+bias), or SwiGLU: the workgroup's two
//    column tiles are the gate rows n and the up rows I+n of the fused [2I, K] weight.
#include "skinny_common.h"
#include "launchers.h"

namespace dllm {

constexpr int EPI_STORE = 0;
constexpr int EPI_SWIGLU = 1;

template <int MT, int NT, int EPI>
__global__ void __launch_bounds__(512, 1) gemm_skinny_kernel(bf16* __restrict__ y, const bf16* __restrict__ x,
                                                             const bf16* __restrict__ w,
                                                             const bf16* __restrict__ bias, int M, int N, int K,
                                                             int ldy, int up_off) {
  constexpr int BM = MT * 16, BN = NT * 16;
  __shared__ __attribute__((aligned(16))) float red[BM * BN];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  for (int i = threadIdx.x; i < BM * BN; i += 512) red[i] = 0.f;

  const bf16* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    int n0;
    if (EPI == EPI_SWIGLU) n0 = (nt < NT / 2 ? 0 : up_off) + blockIdx.x * (BN / 2) + (nt % (NT / 2)) * 16;
    else n0 = blockIdx.x * BN + nt * 16;
    wrow[nt] = w + (size_t)(n0 + r) * K + 8 * g;
  }
  const bf16* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xrow[mt] = x + (size_t)min(mt * 16 + r, M - 1) * K + 8 * g;

  const int ngroups = K >> 7;   // 128-wide k-groups
  const int per = (ngroups + kSkWaves - 1) / kSkWaves;
  const int g0 = wv * per, g1 = min(ngroups, g0 + per);

  f32x4 acc[MT][NT];
  sk_mainloop<MT, NT>(acc, xrow, wrow, g0, g1);
  __syncthreads();   // LDS zero-fill visible
  sk_reduce_lds<MT, NT>(red, acc, lane);
  __syncthreads();

  if (EPI == EPI_SWIGLU) {
    constexpr int HB = BN / 2;   // outputs per workgroup
    for (int e = threadIdx.x; e < M * HB; e += 512) {
      const int m = e / HB, c = e % HB;
      const float gt = red[m * BN + c], up = red[m * BN + HB + c];
      y[(size_t)m * ldy + blockIdx.x * HB + c] = f2bf(silu_f(gt) * up);
    }
  } else {
    for (int e = threadIdx.x; e < M * BN; e += 512) {
      const int m = e / BN, c = e % BN;
      const int n = blockIdx.x * BN + c;
      float v = red[m * BN + c];
      if (bias) v += bf2f(bias[n]);
      y[(size_t)m * ldy + n] = f2bf(v);
    }
  }
}

// NT choice: as many workgroups as possible while >= 512 (2 per CU), else NT = 1.
static int pick_nt(int cols, bool swiglu) {
  if (swiglu) return 2;   // one gate tile + one up tile -> 16 outputs per workgroup
  for (int nt : {4, 2})
    if (cols % (16 * nt) == 0 && cols / (16 * nt) >= 512) return nt;
  return 1;
}

template <int MT, int NT, int EPI>
static void launch_sk(uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t bias, int M, int N, int K, int ldy,
                      int up_off, hipStream_t s) {
  constexpr int BN = NT * 16;
  const int grid = (EPI == EPI_SWIGLU) ? up_off / (BN / 2) : N / BN;
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, NT, EPI>), dim3(grid), dim3(512), 0, s, (bf16*)y, (const bf16*)x,
                     (const bf16*)w, (const bf16*)bias, M, N, K, ldy, up_off);
}

template <int MT>
static void dispatch_mt(uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t bias, int M, int N, int K, int mode,
                        hipStream_t s) {
  if (mode == 1) {
    launch_sk<MT, 2, EPI_SWIGLU>(y, x, w, 0, M, N, K, N / 2, N / 2, s);
    return;
  }
  int nt = pick_nt(N, false);
  if (MT == 4 && nt == 4) nt = 2;   // MT=4 x NT=4 spills (256 VGPRs)
  switch (nt) {
    case 4: launch_sk<(MT < 4 ? MT : 2), 4, EPI_STORE>(y, x, w, bias, M, N, K, N, 0, s); break;
    case 2: launch_sk<MT, 2, EPI_STORE>(y, x, w, bias, M, N, K, N, 0, s); break;
    default: launch_sk<MT, 1, EPI_STORE>(y, x, w, bias, M, N, K, N, 0, s); break;
  }
}

// mode 0: y[M,N] = x W^T (+bias);  mode 1: y[M, N/2] = silu(x Wg^T) * (x Wu^T), W = [Wg; Wu]
void gemm_skinny(uintptr_t y, uintptr_t x, uintptr_t w, uintptr_t bias, int M, int N, int K, int mode,
                 uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1 && M <= 64, "skinny GEMM handles 1 <= M <= 64");
  DLLM_HOST_CHECK(K % 128 == 0, "K must be a multiple of 128");
  DLLM_HOST_CHECK(mode == 0 || mode == 1, "mode");
  if (mode == 1) {
    DLLM_HOST_CHECK(N % 32 == 0, "SwiGLU: N (=2I) must be a multiple of 32");
    DLLM_HOST_CHECK(bias == 0, "SwiGLU: no bias");
  } else {
    DLLM_HOST_CHECK(N % 16 == 0, "N must be a multiple of 16");
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (M <= 16) dispatch_mt<1>(y, x, w, bias, M, N, K, mode, s);
  else if (M <= 32) dispatch_mt<2>(y, x, w, bias, M, N, K, mode, s);
  else dispatch_mt<4>(y, x, w, bias, M, N, K, mode, s);
  DLLM_HIP_CHECK(hipGetLastError());
}

}  // namespace dllm
