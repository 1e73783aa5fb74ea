// Building blocks of the weight-streaming (small-M) MFMA GEMM: the Mixtral grouped expert GEMM
// for few tokens per expert (moe.hip).
//
// v_mfma_f32_16x16x32_bf16 fragments, k permuted inside each 128-wide k-group identically
// for X and W (a dot product is order-invariant): load i of lane (r, g) reads elements
// 32*i + 8*g .. +7 of row r, so ONE wave-instruction reads 64 contiguous bytes of each of
// 16 rows (16 half-lines) rather than 16 B from each of 32 lines (the first layout, 8*i + 32*g),
// halving the lines the texture path touches per instruction.  Row pointers carry the +8*g.
#pragma once
#include "common.h"

namespace dllm {

constexpr int kSkWaves = 8;

template <int MT, int NT>
__device__ __forceinline__ void sk_load(bf16x8 (&xa)[MT][4], bf16x8 (&wb)[NT][4], const bf16* const (&xrow)[MT],
                                        const bf16* const (&wrow)[NT], int k) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(wrow[nt] + k);
#pragma unroll
    for (int i = 0; i < 4; ++i) wb[nt][i] = __builtin_nontemporal_load(p + 4 * i);
  }
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const bf16x8* p = reinterpret_cast<const bf16x8*>(xrow[mt] + k);
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[mt][i] = p[4 * i];
  }
}

template <int MT, int NT>
__device__ __forceinline__ void sk_mma(f32x4 (&acc)[MT][NT], const bf16x8 (&xa)[MT][4], const bf16x8 (&wb)[NT][4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[mt][i], wb[nt][i], acc[mt][nt], 0, 0, 0);
}

// acc[MT][NT] over k-groups [g0, g1) of 128, double-buffered register loads.
template <int MT, int NT>
__device__ __forceinline__ void sk_mainloop(f32x4 (&acc)[MT][NT], const bf16* const (&xrow)[MT],
                                            const bf16* const (&wrow)[NT], int g0, int g1) {
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (g0 >= g1) return;
  bf16x8 xa0[MT][4], wb0[NT][4], xa1[MT][4], wb1[NT][4];
  int gg = g0;
  sk_load<MT, NT>(xa0, wb0, xrow, wrow, gg * 128);
  for (; gg + 1 < g1; gg += 2) {
    sk_load<MT, NT>(xa1, wb1, xrow, wrow, (gg + 1) * 128);
    sk_mma<MT, NT>(acc, xa0, wb0);
    if (gg + 2 < g1) sk_load<MT, NT>(xa0, wb0, xrow, wrow, (gg + 2) * 128);
    sk_mma<MT, NT>(acc, xa1, wb1);
  }
  if (gg < g1) sk_mma<MT, NT>(acc, xa0, wb0);
}

// Sum the 8 waves' partial tiles into red[BM][BN] (zeroed beforehand) with LDS float atomics.
// Sum of the WAVES waves' partial tiles (each wave ran a K slice) into red (zeroed by the caller,
// behind a barrier), wave 0 first, then 1, ...: a fixed order, so the result is the same on every
// run.  (LDS atomicAdd summed them in arrival order: the MoE expert GEMM's bf16 outputs changed
// from run to run, and a pipeline over Mixtral-dims stages disagreed with itself.)  Ends behind a
// barrier.
template <int MT, int NT, int WAVES>
__device__ __forceinline__ void sk_reduce_lds(float* red, const f32x4 (&acc)[MT][NT], int lane, int wv) {
  constexpr int BN = NT * 16;
  const int r = lane & 15, g = lane >> 4;
#pragma unroll 1
  for (int w = 0; w < WAVES; ++w) {
    if (wv == w) {
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
          for (int i = 0; i < 4; ++i) red[(mt * 16 + 4 * g + i) * BN + nt * 16 + r] += acc[mt][nt][i];
    }
    __syncthreads();
  }
}

}  // namespace dllm
