// Dynamic per-token FP8 quantization for the W8A8 decode GEMMs (gemm_wide_fp8).
//
// Row m of x [M, K] bf16 -> q [M, K] OCP e4m3 (gfx950's FP8 format, not MI300's fnuz) and
// scale[m] = amax(|x_m|) / 448 (448 = the largest finite e4m3), q = RNE(x / scale).  One
// 256-thread workgroup per row, the row held in registers between the max and the convert pass
// (MAXV 16-byte vectors per thread; MAXV = 0 re-reads the row for K > 16384), packed conversions
// (v_cvt_pk_fp8_f32) and 8-byte stores.  The GEMM multiplies its accumulator by
// scale[m] * wscale[n] in the epilogue.  The RMSNorm kernels carry the same epilogue (q8 output)
// for the projections that follow a norm; this kernel serves the o and down projection inputs.
#include "common.h"
#include "launchers.h"

namespace dllm {

template <int MAXV>
__global__ void __launch_bounds__(256) quant_fp8_rows_kernel(uint8_t* __restrict__ q, float* __restrict__ scale,
                                                             const bf16* __restrict__ x, int K) {
  __shared__ float red[16];
  const int m = blockIdx.x, tid = threadIdx.x;
  const int nvec = K >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)m * K);
  uint8_t* qr = q + (size_t)m * K;
  float amax = 0.f;
  if constexpr (MAXV > 0) {
    float v[MAXV][8];
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int idx = tid + i * 256;
      if (idx < nvec) {
        const bf16x8 a = xr[idx];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[i][j] = bf2f(a[j]);
          amax = fmaxf(amax, fabsf(v[i][j]));
        }
      }
    }
    const float s = fp8_row_scale(block_max(amax, red));
    if (tid == 0) scale[m] = s;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const int idx = tid + i * 256;
      if (idx < nvec) store8_fp8(qr + idx * 8, v[i], s);
    }
  } else {
    for (int idx = tid; idx < nvec; idx += 256) {
      const bf16x8 a = xr[idx];
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(a[j])));
    }
    const float s = fp8_row_scale(block_max(amax, red));
    if (tid == 0) scale[m] = s;
    for (int idx = tid; idx < nvec; idx += 256) {
      const bf16x8 a = xr[idx];
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = bf2f(a[j]);
      store8_fp8(qr + idx * 8, v, s);
    }
  }
}

void quant_fp8_rows(uintptr_t q, uintptr_t scale, uintptr_t x, int M, int K, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(K % 8 == 0 && K >= 8, "K must be a positive multiple of 8");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nvec = K / 8;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(M), dim3(256), 0, s, (uint8_t*)q, (float*)scale, (const bf16*)x, K);
  };
  if (nvec <= 256) go(quant_fp8_rows_kernel<1>);
  else if (nvec <= 512) go(quant_fp8_rows_kernel<2>);
  else if (nvec <= 1024) go(quant_fp8_rows_kernel<4>);
  else if (nvec <= 2048) go(quant_fp8_rows_kernel<8>);
  else go(quant_fp8_rows_kernel<0>);
  DLLM_HIP_CHECK(hipGetLastError());
}

}  // namespace dllm
