// Split-K slab consumers: every split-K GEMM (gemm_wide / gemm_sq / gemm_pp, MoE) leaves S partial
// slabs (f16 x 2^-6 by default, common.h DLLM_PART_TYPE) in the per-stream workspace; these kernels
// turn them into the next op's input without another round trip:
//  * splitk_add_rms_norm(_q8): reduce + residual add + RMSNorm (+ per-token e4m3 for a W8A8 GEMM),
//    the o / down projections' epilogue in every Llama block;
//  * splitk_reduce(_ex): plain reduce (+bias) or reduce + SwiGLU.
// Slab counts 2..8 are compile-time instantiations: all of a vector's slab loads are in flight
// before the first add (nontemporal: slabs are read once).
#include "common.h"
#include "launchers.h"

namespace dllm {

// out[m, n] = sum_s P[s, m, n] (+ bias[n]);  swiglu: out[m, j] = silu(sum P[m, j]) * sum P[m, I + j]
template <bool SWIGLU, int SC>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16* __restrict__ out, const float* __restrict__ P,
                                                            const bf16* __restrict__ bias, int S_, int M, int N) {
  // SC > 0: compile-time slab count -> every slab load of a vector is in flight before the first
  // add (nontemporal: the slabs are read once); SC == 0: runtime loop
  const int S = SC > 0 ? SC : S_;
  const int ncols = SWIGLU ? N / 2 : N;
  const long total = (long)M * ncols / 4;
  const size_t slab = (size_t)M * N;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const long e = v * 4;
    const int m = (int)(e / ncols), c = (int)(e % ncols);
    f32x4 a = {0.f, 0.f, 0.f, 0.f}, u = {0.f, 0.f, 0.f, 0.f};
    if constexpr (SC > 0) {
      f32x4 la[SC], lu[SC];
#pragma unroll
      for (int s = 0; s < SC; ++s) {
        la[s] = part_load4<true>(P, s * slab + (size_t)m * N + c);
        if (SWIGLU) lu[s] = part_load4<true>(P, s * slab + (size_t)m * N + ncols + c);
      }
#pragma unroll
      for (int s = 0; s < SC; ++s) {   // same slab order as the runtime loop: bit-identical sums
        a += la[s];
        if (SWIGLU) u += lu[s];
      }
    } else {
      for (int s = 0; s < S; ++s) {
        a += part_load4(P, s * slab + (size_t)m * N + c);
        if (SWIGLU) u += part_load4(P, s * slab + (size_t)m * N + ncols + c);
      }
    }
    bf16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float x = a[j];
      if (SWIGLU) x = silu_f(x) * u[j];
      else if (bias) x += bf2f(bias[c + j]);
      o[j] = f2bf(x);
    }
    *reinterpret_cast<bf16x4*>(out + (size_t)m * ncols + c) = o;
  }
}

// Split-K reduce fused into the NEXT op of a Llama block: residual add + RMSNorm.
//   h = bf16(sum_s P[s, row, :]);  r = bf16(h + residual);  residual <- r;  y = rmsnorm(r) * w
// Bit-identical to splitk_reduce_kernel followed by rms_norm_kernel with a residual (same
// per-element summation order, same thread -> vector mapping for the sum of squares), minus one
// launch and the bf16 h round trip through HBM.  One 256-thread workgroup per row.
template <int MAXV, int SC, int NTH = 256>
__global__ void __launch_bounds__(NTH) splitk_add_rms_norm_kernel(bf16* __restrict__ y, bf16* __restrict__ residual,
                                                                  const float* __restrict__ P, int S_, int M, int N,
                                                                  const bf16* __restrict__ w, float eps,
                                                                  uint8_t* __restrict__ q8, float* __restrict__ qs) {
  // SC > 0: the slab count is a compile-time constant, so all of a vector's 2*SC slab loads are
  // issued before the first add (the runtime-S loop waited on each slab in turn)
  const int S = SC > 0 ? SC : S_;
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = N >> 3;
  const size_t slab = (size_t)M * N;
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + (size_t)row * N);
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * NTH;
    if (idx < nvec) {
      const size_t p = (size_t)row * N + idx * 8;
      f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
      if constexpr (SC > 0) {
        f32x4 l0[SC], l1[SC];
#pragma unroll
        for (int s = 0; s < SC; ++s) {
          l0[s] = part_load4<true>(P, p + s * slab);
          l1[s] = part_load4<true>(P, p + s * slab + 4);
        }
#pragma unroll
        for (int s = 0; s < SC; ++s) {   // same slab order as the runtime loop: bit-identical sums
          a0 += l0[s];
          a1 += l1[s];
        }
      } else {
        for (int s = 0; s < S; ++s) {
          a0 += part_load4(P, p + s * slab);
          a1 += part_load4(P, p + s * slab + 4);
        }
      }
      const bf16x8 b = rr[idx];
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = bf2f(f2bf(j < 4 ? a0[j] : a1[j - 4]));
        r[j] = f2bf(h + bf2f(b[j]));
      }
      rr[idx] = r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f(r[j]);
        ss += v[i][j] * v[i][j];
      }
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)N + eps);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  if (q8) {   // FP8 consumer: per-token e4m3 of the normalised row (rms_norm_kernel's epilogue)
    norm_out_fp8<MAXV, NTH>(v, inv, wv, nvec, y ? y + (size_t)row * N : nullptr, q8 + (size_t)row * N, qs + row,
                            red);
    return;
  }
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)row * N);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * NTH;
    if (idx < nvec) {
      const bf16x8 g = wv[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
      yr[idx] = o;
    }
  }
}

void splitk_add_rms_norm(uintptr_t y, uintptr_t residual, uintptr_t ws, int S, int M, int N, uintptr_t w, float eps,
                         uintptr_t stream) {
  splitk_add_rms_norm_q8(y, residual, ws, S, M, N, w, eps, 0, 0, stream);
}

void splitk_add_rms_norm_q8(uintptr_t y, uintptr_t residual, uintptr_t ws, int S, int M, int N, uintptr_t w,
                            float eps, uintptr_t q8, uintptr_t qs, uintptr_t stream) {
  DLLM_HOST_CHECK(N % 8 == 0 && N <= 8 * 256 * 8, "hidden must be a multiple of 8 and <= 16384");
  DLLM_HOST_CHECK(y != 0 || q8 != 0, "splitk_add_rms_norm needs an output");
  DLLM_HOST_CHECK((q8 == 0) == (qs == 0), "q8 and its scales go together");
  DLLM_HOST_CHECK(S >= 1 && M >= 0, "S >= 1");
  if (M == 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(M), dim3(256), 0, s, (bf16*)y, (bf16*)residual, (const float*)ws, S, M, N,
                       (const bf16*)w, eps, (uint8_t*)q8, (float*)qs);
  };
  const int nvec = N / 8;
#define DLLM_SKN(MV)                                                   \
  do {                                                                 \
    if (S == 8) go(splitk_add_rms_norm_kernel<MV, 8>);                 \
    else if (S == 4) go(splitk_add_rms_norm_kernel<MV, 4>);            \
    else if (S == 2) go(splitk_add_rms_norm_kernel<MV, 2>);            \
    else if (S == 3) go(splitk_add_rms_norm_kernel<MV, 3>);            \
    else if (S == 5) go(splitk_add_rms_norm_kernel<MV, 5>);            \
    else if (S == 6) go(splitk_add_rms_norm_kernel<MV, 6>);            \
    else if (S == 7) go(splitk_add_rms_norm_kernel<MV, 7>);            \
    else go(splitk_add_rms_norm_kernel<MV, 0>);                        \
  } while (0)
  if (nvec <= 256) DLLM_SKN(1);
  else if (nvec <= 512) DLLM_SKN(2);
  else if (nvec <= 1024) DLLM_SKN(4);
  else DLLM_SKN(8);
#undef DLLM_SKN
  DLLM_HIP_CHECK(hipGetLastError());
}

// plain split-K reduce of the partial slabs a split GEMM left (mode 2 of gemm_wide / gemm_sq / gemm_pp): out = bf16(sum_s P[s]) (+bias)
void splitk_reduce_ex(uintptr_t out, uintptr_t ws, uintptr_t bias, int S, int M, int N, int swiglu,
                      uintptr_t stream) {
  DLLM_HOST_CHECK(N % (swiglu ? 8 : 4) == 0, "N alignment");
  const int ncols = swiglu ? N / 2 : N;
  long blocks = ((long)M * ncols / 4 + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bf16* b = swiglu ? nullptr : (const bf16*)bias;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, (bf16*)out, (const float*)ws, b, S, M, N);
  };
#define DLLM_SKR(SW)                                                   \
  do {                                                                 \
    switch (S) {                                                       \
      case 2: go(splitk_reduce_kernel<SW, 2>); break;                  \
      case 3: go(splitk_reduce_kernel<SW, 3>); break;                  \
      case 4: go(splitk_reduce_kernel<SW, 4>); break;                  \
      case 5: go(splitk_reduce_kernel<SW, 5>); break;                  \
      case 6: go(splitk_reduce_kernel<SW, 6>); break;                  \
      case 8: go(splitk_reduce_kernel<SW, 8>); break;                  \
      default: go(splitk_reduce_kernel<SW, 0>);                        \
    }                                                                  \
  } while (0)
  if (swiglu) DLLM_SKR(true); else DLLM_SKR(false);
#undef DLLM_SKR
  DLLM_HIP_CHECK(hipGetLastError());
}

void splitk_reduce(uintptr_t out, uintptr_t ws, uintptr_t bias, int S, int M, int N, uintptr_t stream) {
  splitk_reduce_ex(out, ws, bias, S, M, N, 0, stream);
}

}  // namespace dllm
