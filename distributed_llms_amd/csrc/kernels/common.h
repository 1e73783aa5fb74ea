// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels.
//
// Wave = 64 lanes (never 32). bf16 is the storage type everywhere; math is f32.
// Vector types match MFMA operand registers: 8 x bf16 = 4 VGPRs per lane.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define DLLM_WAVE 64

#define DLLM_HOST_CHECK(cond, msg)                                                     \
  do {                                                                                 \
    if (!(cond)) throw std::runtime_error(std::string("dllm kernel precondition: ") + \
                                          (msg) + " [" #cond "]");                     \
  } while (0)

#define DLLM_HIP_CHECK(expr)                                                           \
  do {                                                                                 \
    hipError_t _e = (expr);                                                            \
    if (_e != hipSuccess)                                                              \
      throw std::runtime_error(std::string("HIP error: ") + hipGetErrorString(_e) +    \
                               " at " __FILE__ ":" + std::to_string(__LINE__));         \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, DLLM_WAVE);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, DLLM_WAVE));
  return v;
}

// Reduction over a lane's xor-16 and xor-32 partners (the four 16-lane rows of an MFMA 16x16
// accumulator column) with the gfx950 VALU row swaps instead of __shfl_xor, which lowers to two
// dependent ds_bpermute LDS round trips.  v_permlane16_swap(x, x) leaves rows (0, 0, 2, 2) in the
// first result and (1, 1, 3, 3) in the second, v_permlane32_swap(x, x) halves (lo, lo) / (hi, hi):
// combining the pair is the butterfly step.  Bit-identical to the shuffle form (max and a
// two-operand add commute).
__device__ __forceinline__ float rows_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float rows_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Block-wide sum for blockDim.x <= 1024; `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  __syncthreads();
  return t;
}

// SiLU with the hardware reciprocal (v_rcp_f32, 1 ulp): hipcc expands x / y into the IEEE division
// sequence (2 v_div_scale, v_rcp, 4 FMAs, v_div_fmas, v_div_fixup), which made gemm_pf's SwiGLU
// epilogue ~2,200 VALU per 256x256 tile per wave with the MFMA pipe idle; every caller rounds the
// result to bf16
__device__ __forceinline__ float silu_f(float x) { return x * __builtin_amdgcn_rcpf(1.f + __expf(-x)); }

// f32 -> bf16 via the compiler cast: gfx950 emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }
__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }

// Block-wide max for blockDim.x <= 1024; `red` must hold >= 16 floats.
__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = wave_max(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = red[0];
  for (int i = 1; i < nw; ++i) t = fmaxf(t, red[i]);
  __syncthreads();
  return t;
}

// ---- per-token FP8 (OCP e4m3) quantization shared by quant.hip and the fused norm epilogues:
// scale = amax / 448 (1 for an all-zero row), q = RNE(clamp(v / scale)), packed 4 per dword.
constexpr float kFp8Max = 448.f;
__device__ __forceinline__ float fp8_row_scale(float amax) { return amax > 0.f ? amax / kFp8Max : 1.f; }
__device__ __forceinline__ float fp8_in(float v, float s) { return fminf(fmaxf(v / s, -kFp8Max), kFp8Max); }
__device__ __forceinline__ int pack4_fp8(float a, float b, float c, float d) {
  int w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
// 8 values (already bf16-rounded, in f32) -> 8 e4m3 bytes at q
__device__ __forceinline__ void store8_fp8(uint8_t* q, const float (&v)[8], float s) {
  int2 o;
  o.x = pack4_fp8(fp8_in(v[0], s), fp8_in(v[1], s), fp8_in(v[2], s), fp8_in(v[3], s));
  o.y = pack4_fp8(fp8_in(v[4], s), fp8_in(v[5], s), fp8_in(v[6], s), fp8_in(v[7], s));
  *reinterpret_cast<int2*>(q) = o;
}

// Norm epilogue with an FP8 consumer: y = bf16(v * inv * g) per element (written when y != null),
// then the row's e4m3 quantization of those bf16 values (q8 row, scale at *qs).  v [MAXV][8]: the
// thread's row values, vector idx = threadIdx.x + i * NTH.
template <int MAXV, int NTH>
__device__ __forceinline__ void norm_out_fp8(float (&v)[MAXV][8], float inv, const bf16x8* __restrict__ wv, int nvec,
                                             bf16* __restrict__ y, uint8_t* __restrict__ q8, float* __restrict__ qs,
                                             float* red) {
  float amax = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * NTH;
    if (idx < nvec) {
      const bf16x8 g = wv[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
        v[i][j] = bf2f(o[j]);
        amax = fmaxf(amax, fabsf(v[i][j]));
      }
      if (y) reinterpret_cast<bf16x8*>(y)[idx] = o;
    }
  }
  const float s = fp8_row_scale(block_max(amax, red));
  if (threadIdx.x == 0) *qs = s;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * NTH;
    if (idx < nvec) store8_fp8(q8 + idx * 8, v[i], s);
  }
}

// Paged KV layout of a 32-key block (one kv head), chosen so that the QK^T MFMA output hands
// every lane group g the probabilities of keys 8g..8g+7 in natural order:
//   K  [32 rows][D]        key j stored at row krow32(j): 8g+i -> row 4g+i, 8g+4+i -> row 16+4g+i
//                          (rows 0-15 / 16-31 are the two 16-key MFMA tiles; lane group g of the
//                          S^T = K Q^T result holds rows 4g..4g+3 of each tile = keys 8g..8g+7)
//   V^T [4][D][8]          element (key j, dim d) at (j/8)*8D + 8d + j%8: the P.V A-fragment of
//                          lane (dim d, group g) -- keys 8g..8g+7 of dim d -- is one 16-byte load,
//                          and a new token's 128 dims land in one 2 KiB span (16 cache lines, not
//                          64: the per-step append dirties 4x fewer partial lines)
// Other block sizes (CPU reference path only) use plain rows / a plain [D][bs] V^T.
__host__ __device__ __forceinline__ int krow32(int j) { return ((j & 4) << 2) + ((j >> 3) << 2) + (j & 3); }
__host__ __device__ __forceinline__ int krow(int off, int bs) { return bs == 32 ? krow32(off) : off; }
// element offset of (key off, dim e) inside one head's V^T block of bs keys x d dims
__host__ __device__ __forceinline__ int vofs(int off, int e, int d, int bs) {
  return bs == 32 ? (off >> 3) * 8 * d + e * 8 + (off & 7) : e * bs + off;
}

// ---- split-K partial slabs (the workspace the split GEMMs leave for the next op).
// DLLM_PART_TYPE selects the slab element (indices are in elements of that type):
//   0  f32
//   1  bf16           (8-bit significand: the test tolerances of a 14k-deep sum are exceeded)
//   2  f16 x 2^-6     (default: 11-bit significand, 3 bits more than the bf16 output; the 2^-6
//                      scale puts the f16 range at +-4.2e6 and the subnormal step at 3.8e-6)
// Each K slice still accumulates in f32 MFMA registers and the cross-slice sum is f32; 2 and 1
// halve the slab bytes the GEMM epilogue writes and the next op reads.
#ifndef DLLM_PART_TYPE
#define DLLM_PART_TYPE 2
#endif
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
constexpr float kPartScale = 0.015625f, kPartUnscale = 64.f;
__device__ __forceinline__ void part_store(float* P, size_t i, float v) {
#if DLLM_PART_TYPE == 1
  reinterpret_cast<bf16*>(P)[i] = f2bf(v);
#elif DLLM_PART_TYPE == 2
  reinterpret_cast<_Float16*>(P)[i] = (_Float16)(v * kPartScale);
#else
  P[i] = v;
#endif
}
__device__ __forceinline__ float part_load1(const float* P, size_t i) {
#if DLLM_PART_TYPE == 1
  return bf2f(reinterpret_cast<const bf16*>(P)[i]);
#elif DLLM_PART_TYPE == 2
  return (float)reinterpret_cast<const _Float16*>(P)[i] * kPartUnscale;
#else
  return P[i];
#endif
}
// 4 consecutive elements (aligned to 4 elements)
template <bool NT = false>
__device__ __forceinline__ f32x4 part_load4(const float* P, size_t i) {
#if DLLM_PART_TYPE == 1
  const bf16x4* q = reinterpret_cast<const bf16x4*>(reinterpret_cast<const bf16*>(P) + i);
  const bf16x4 v = NT ? __builtin_nontemporal_load(q) : *q;
  return f32x4{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
#elif DLLM_PART_TYPE == 2
  const f16x4* q = reinterpret_cast<const f16x4*>(reinterpret_cast<const _Float16*>(P) + i);
  const f16x4 v = NT ? __builtin_nontemporal_load(q) : *q;
  return f32x4{(float)v[0], (float)v[1], (float)v[2], (float)v[3]} * kPartUnscale;
#else
  const f32x4* q = reinterpret_cast<const f32x4*>(P + i);
  return NT ? __builtin_nontemporal_load(q) : *q;
#endif
}
