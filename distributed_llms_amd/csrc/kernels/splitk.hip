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
// Each thread reduces V = 8 consecutive outputs (16-byte slab loads; 4 where ncols % 8 != 0).
template <bool SWIGLU, int SC, int V>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(bf16* __restrict__ out, const float* __restrict__ P,
                                                            const bf16* __restrict__ bias, int S_, int M, int N) {
  // SC > 0: compile-time slab count -> every slab load of a vector is in flight before the first
  // add (nontemporal: the slabs are read once); SC == 0: runtime loop
  static_assert(V == 4 || V == 8, "4 or 8 outputs per thread");
  constexpr int H = V / 4;
  const int S = SC > 0 ? SC : S_;
  const int ncols = SWIGLU ? N / 2 : N;
  const long total = (long)M * ncols / V;
  const size_t slab = (size_t)M * N;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < total; v += (long)gridDim.x * 256) {
    const long e = v * V;
    const int m = (int)(e / ncols), c = (int)(e % ncols);
    const size_t p = (size_t)m * N + c;
    f32x4 a[H], u[H];
#pragma unroll
    for (int h = 0; h < H; ++h) a[h] = u[h] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (SC > 0) {
      f32x4 la[SC][H], lu[SC][H];
#pragma unroll
      for (int s = 0; s < SC; ++s) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
          la[s][h] = part_load4<true>(P, s * slab + p + 4 * h);
          if (SWIGLU) lu[s][h] = part_load4<true>(P, s * slab + p + ncols + 4 * h);
        }
      }
#pragma unroll
      for (int s = 0; s < SC; ++s) {   // same slab order as the runtime loop: bit-identical sums
#pragma unroll
        for (int h = 0; h < H; ++h) {
          a[h] += la[s][h];
          if (SWIGLU) u[h] += lu[s][h];
        }
      }
    } else {
      for (int s = 0; s < S; ++s) {
#pragma unroll
        for (int h = 0; h < H; ++h) {
          a[h] += part_load4(P, s * slab + p + 4 * h);
          if (SWIGLU) u[h] += part_load4(P, s * slab + p + ncols + 4 * h);
        }
      }
    }
    bf16x4 o[H];
#pragma unroll
    for (int h = 0; h < H; ++h) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float x = a[h][j];
        if (SWIGLU) x = silu_f(x) * u[h][j];
        else if (bias) x += bf2f(bias[c + 4 * h + j]);
        o[h][j] = f2bf(x);
      }
    }
    bf16* dst = out + (size_t)m * ncols + c;
    if constexpr (V == 8) {
      bf16x8 o8;
#pragma unroll
      for (int j = 0; j < 8; ++j) o8[j] = o[j >> 2][j & 3];
      *reinterpret_cast<bf16x8*>(dst) = o8;
    } else {
      *reinterpret_cast<bf16x4*>(dst) = o[0];
    }
  }
}

// Split-K reduce fused into the NEXT op of a Llama block: residual add + RMSNorm.
//   h = bf16(sum_s P[s, row, :]);  r = bf16(h + residual);  residual <- r;  y = rmsnorm(r) * w
// Bit-identical to splitk_reduce_kernel followed by rms_norm_kernel with a residual (same
// per-element summation order, same thread -> vector mapping for the sum of squares), minus one
// launch and the bf16 h round trip through HBM.  One 256-thread workgroup per row.
template <int MAXV, int SC, bool EX, int NTH = 256>
__global__ void __launch_bounds__(NTH) splitk_add_rms_norm_kernel(bf16* __restrict__ y, bf16* __restrict__ residual,
                                                                  const float* __restrict__ P, int S_, int M, int N,
                                                                  const bf16* __restrict__ w, float eps,
                                                                  uint8_t* __restrict__ q8, float* __restrict__ qs) {
  // SC > 0: the slab count is a compile-time constant, so all of a vector's 2*SC slab loads are
  // issued before the first add (the runtime-S loop waited on each slab in turn)
  //
  // Every global load of the row -- slabs, residual AND the norm weight -- is issued before the
  // first use, in chunks of CH vectors (<= 32 slab loads in flight per thread), off clamped vector
  // ids.  EX (N == 8 * MAXV * NTH, e.g. 4096 / 8192): no per-lane guard at all.  Behind a guard
  // (idx < nvec) hipcc sank each vector's loads into its own branch, waiting for vector i's slabs
  // before issuing vector i + 1's, and fetched the weight only after the block sum: three
  // dependent memory round trips instead of one.
  const int S = SC > 0 ? SC : S_;
  constexpr int SE = SC > 0 ? SC : 1;
  constexpr int CH = MAXV * SE <= 16 ? MAXV : (16 / SE > 0 ? 16 / SE : 1);
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = N >> 3;
  const size_t slab = (size_t)M * N;
  bf16x8* rr = reinterpret_cast<bf16x8*>(residual + (size_t)row * N);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  float v[MAXV][8];
  bf16x8 g[MAXV];
  float ss = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) g[k] = wv[min((int)threadIdx.x + k * NTH, nvec - 1)];
#pragma unroll
  for (int c0 = 0; c0 < MAXV; c0 += CH) {
    f32x4 a0[CH], a1[CH];
    bf16x8 b[CH];
    if constexpr (SC > 0) {
      f32x4 l0[CH][SC], l1[CH][SC];
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int idc = min((int)threadIdx.x + (c0 + i) * NTH, nvec - 1);
        const size_t p = (size_t)row * N + idc * 8;
#pragma unroll
        for (int s = 0; s < SC; ++s) {
          l0[i][s] = part_load4<true>(P, p + s * slab);
          l1[i][s] = part_load4<true>(P, p + s * slab + 4);
        }
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int idc = min((int)threadIdx.x + (c0 + i) * NTH, nvec - 1);
        b[i] = rr[idc];
      }
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        a0[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        a1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < SC; ++s) {   // same slab order as the runtime loop: bit-identical sums
          a0[i] += l0[i][s];
          a1[i] += l1[i][s];
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        const int idc = min((int)threadIdx.x + (c0 + i) * NTH, nvec - 1);
        const size_t p = (size_t)row * N + idc * 8;
        b[i] = rr[idc];
        a0[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        a1[i] = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int s = 0; s < S; ++s) {
          a0[i] += part_load4(P, p + s * slab);
          a1[i] += part_load4(P, p + s * slab + 4);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      const int idx = threadIdx.x + (c0 + i) * NTH;
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float h = bf2f(f2bf(j < 4 ? a0[i][j] : a1[i][j - 4]));
        r[j] = f2bf(h + bf2f(b[i][j]));
      }
      if (EX || idx < nvec) {
        rr[idx] = r;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[c0 + i][j] = bf2f(r[j]);
          ss += v[c0 + i][j] * v[c0 + i][j];
        }
      }
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)N + eps);
  if (q8) {   // FP8 consumer: per-token e4m3 of the normalised row (rms_norm_kernel's epilogue)
    norm_out_fp8<MAXV, NTH>(v, inv, wv, nvec, y ? y + (size_t)row * N : nullptr, q8 + (size_t)row * N, qs + row,
                            red);
    return;
  }
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)row * N);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * NTH;
    if (EX || idx < nvec) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[i][j]));
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
#define DLLM_SKN2(MV, EX)                                              \
  do {                                                                 \
    if (S == 8) go(splitk_add_rms_norm_kernel<MV, 8, EX>);             \
    else if (S == 4) go(splitk_add_rms_norm_kernel<MV, 4, EX>);        \
    else if (S == 2) go(splitk_add_rms_norm_kernel<MV, 2, EX>);        \
    else if (S == 3) go(splitk_add_rms_norm_kernel<MV, 3, EX>);        \
    else if (S == 5) go(splitk_add_rms_norm_kernel<MV, 5, EX>);        \
    else if (S == 6) go(splitk_add_rms_norm_kernel<MV, 6, EX>);        \
    else if (S == 7) go(splitk_add_rms_norm_kernel<MV, 7, EX>);        \
    else go(splitk_add_rms_norm_kernel<MV, 0, EX>);                    \
  } while (0)
#define DLLM_SKN(MV)                                                   \
  do {                                                                 \
    if (nvec == (MV) * 256) DLLM_SKN2(MV, true);                       \
    else DLLM_SKN2(MV, false);                                         \
  } while (0)
  if (nvec <= 256) DLLM_SKN(1);
  else if (nvec <= 512) DLLM_SKN(2);
  else if (nvec <= 1024) DLLM_SKN(4);
  else DLLM_SKN(8);
#undef DLLM_SKN
#undef DLLM_SKN2
  DLLM_HIP_CHECK(hipGetLastError());
}

// plain split-K reduce of the partial slabs a split GEMM left (mode 2 of gemm_wide / gemm_sq / gemm_pp): out = bf16(sum_s P[s]) (+bias)
void splitk_reduce_ex(uintptr_t out, uintptr_t ws, uintptr_t bias, int S, int M, int N, int swiglu,
                      uintptr_t stream) {
  DLLM_HOST_CHECK(N % (swiglu ? 8 : 4) == 0, "N alignment");
  const int ncols = swiglu ? N / 2 : N;
  const bool v8 = ncols % 8 == 0;
  long blocks = ((long)M * ncols / (v8 ? 8 : 4) + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  if (blocks == 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const bf16* b = swiglu ? nullptr : (const bf16*)bias;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(256), 0, st, (bf16*)out, (const float*)ws, b, S, M, N);
  };
#define DLLM_SKR2(SW, V)                                               \
  do {                                                                 \
    switch (S) {                                                       \
      case 2: go(splitk_reduce_kernel<SW, 2, V>); break;               \
      case 3: go(splitk_reduce_kernel<SW, 3, V>); break;               \
      case 4: go(splitk_reduce_kernel<SW, 4, V>); break;               \
      case 5: go(splitk_reduce_kernel<SW, 5, V>); break;               \
      case 6: go(splitk_reduce_kernel<SW, 6, V>); break;               \
      case 8: go(splitk_reduce_kernel<SW, 8, V>); break;               \
      default: go(splitk_reduce_kernel<SW, 0, V>);                     \
    }                                                                  \
  } while (0)
#define DLLM_SKR(SW)                                                   \
  do {                                                                 \
    if (v8) DLLM_SKR2(SW, 8); else DLLM_SKR2(SW, 4);                   \
  } while (0)
  if (swiglu) DLLM_SKR(true); else DLLM_SKR(false);
#undef DLLM_SKR
#undef DLLM_SKR2
  DLLM_HIP_CHECK(hipGetLastError());
}

void splitk_reduce(uintptr_t out, uintptr_t ws, uintptr_t bias, int S, int M, int N, uintptr_t stream) {
  splitk_reduce_ex(out, ws, bias, S, M, N, 0, stream);
}

}  // namespace dllm
