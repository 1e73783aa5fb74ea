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

__device__ __forceinline__ float silu_f(float x) { return x / (1.f + __expf(-x)); }

// f32 -> bf16 via the compiler cast: gfx950 emits v_cvt_pk_bf16_f32 (RNE, NaN-preserving).
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }
__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }

// Paged V^T cache, 32-key blocks: key j of a block row is stored at column vperm32(j), order
// 0-3,16-19,4-7,20-23,...  The P.V MFMA's A fragment of lane group g is keys 4g..4g+3 and
// 16+4g..16+4g+3, which this places in 16 contiguous bytes: one 16-B load per fragment
// instead of two 8-B loads.  Other block sizes are stored unpermuted.
__host__ __device__ __forceinline__ int vperm32(int j) {
  return j < 16 ? ((j >> 2) << 3) + (j & 3) : (((j - 16) >> 2) << 3) + 4 + (j & 3);
}
__host__ __device__ __forceinline__ int vcol(int off, int bs) { return bs == 32 ? vperm32(off) : off; }
