// Memory-bound per-token kernels (K1, K2, K4/K5, SwiGLU activation, argmax).
//
// All of these move bf16 through 16-byte (bf16x8) vectors: hipcc does not
// vectorize bf16 scalar loads (CDNA guide Guideline 13) and scalar bf16 costs
// ~2x on HBM-bound kernels.
#include "common.h"
#include "launchers.h"

namespace dllm {

// ---------------------------------------------------------------------------
// K2: RMSNorm, optionally fused with the residual add.
//   residual == nullptr : y = rmsnorm(x) * w
//   residual != nullptr : r = x + residual; residual <- r; y = rmsnorm(r) * w
// One 256-thread workgroup per row; the row stays in registers between the
// sum-of-squares pass and the scale pass (MAXV vectors of 8 per thread).
// ---------------------------------------------------------------------------
template <int MAXV>
__global__ void __launch_bounds__(256) rms_norm_kernel(bf16* __restrict__ y, const bf16* __restrict__ x,
                                                       bf16* __restrict__ residual,
                                                       const bf16* __restrict__ w, int hidden,
                                                       float eps, uint8_t* __restrict__ q8, float* __restrict__ qs) {
  __shared__ float red[16];
  const int row = blockIdx.x;
  const int nvec = hidden >> 3;
  const bf16x8* xr = reinterpret_cast<const bf16x8*>(x + (size_t)row * hidden);
  bf16x8* rr = residual ? reinterpret_cast<bf16x8*>(residual + (size_t)row * hidden) : nullptr;
  float v[MAXV][8];
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * 256;
    if (idx < nvec) {
      bf16x8 a = xr[idx];
      if (rr) {
        bf16x8 b = rr[idx];
        bf16x8 s;
#pragma unroll
        for (int j = 0; j < 8; ++j) s[j] = f2bf(bf2f(a[j]) + bf2f(b[j]));
        rr[idx] = s;
        a = s;  // normalise the bf16-rounded residual, as the reference does
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[i][j] = bf2f(a[j]);
        ss += v[i][j] * v[i][j];
      }
    }
  }
  ss = block_sum(ss, red);
  const float inv = rsqrtf(ss / (float)hidden + eps);
  const bf16x8* wv = reinterpret_cast<const bf16x8*>(w);
  if (q8) {   // FP8 consumer (W8A8 GEMM): per-token e4m3 of the bf16-rounded output, y optional
    norm_out_fp8<MAXV, 256>(v, inv, wv, nvec, y ? y + (size_t)row * hidden : nullptr, q8 + (size_t)row * hidden,
                            qs + row, red);
    return;
  }
  bf16x8* yr = reinterpret_cast<bf16x8*>(y + (size_t)row * hidden);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int idx = threadIdx.x + i * 256;
    if (idx < nvec) {
      bf16x8 g = wv[idx];
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = f2bf(v[i][j] * inv * bf2f(g[j]));
      yr[idx] = o;
    }
  }
}

void rms_norm(uintptr_t y, uintptr_t x, uintptr_t residual, uintptr_t w, int rows, int hidden,
              float eps, uintptr_t stream) {
  rms_norm_q8(y, x, residual, w, rows, hidden, eps, 0, 0, stream);
}

// q8 != 0: also (y == 0: only) the per-token e4m3 quantization of the output, scales in qs
void rms_norm_q8(uintptr_t y, uintptr_t x, uintptr_t residual, uintptr_t w, int rows, int hidden, float eps,
                 uintptr_t q8, uintptr_t qs, uintptr_t stream) {
  DLLM_HOST_CHECK(hidden % 8 == 0 && hidden <= 8 * 256 * 8, "hidden must be a multiple of 8 and <= 16384");
  DLLM_HOST_CHECK(rows >= 0, "rows >= 0");
  DLLM_HOST_CHECK(y != 0 || q8 != 0, "rms_norm needs an output");
  DLLM_HOST_CHECK((q8 == 0) == (qs == 0), "q8 and its scales go together");
  if (rows == 0) return;
  const int nvec = hidden / 8;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(rows), dim3(256), 0, s, (bf16*)y, (const bf16*)x, (bf16*)residual,
                       (const bf16*)w, hidden, eps, (uint8_t*)q8, (float*)qs);
  };
  if (nvec <= 256) args(rms_norm_kernel<1>);
  else if (nvec <= 512) args(rms_norm_kernel<2>);
  else if (nvec <= 1024) args(rms_norm_kernel<4>);
  else args(rms_norm_kernel<8>);
  DLLM_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// K1: embedding gather. One workgroup per token, 16 B per lane.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) embedding_kernel(bf16* __restrict__ out, const int32_t* __restrict__ ids,
                                                        const bf16* __restrict__ table, int hidden, int vocab) {
  const int t = blockIdx.x;
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);  // clamp: never read outside the table
  const bf16x8* src = reinterpret_cast<const bf16x8*>(table + (size_t)id * hidden);
  bf16x8* dst = reinterpret_cast<bf16x8*>(out + (size_t)t * hidden);
  for (int i = threadIdx.x; i < (hidden >> 3); i += 256) dst[i] = src[i];
}

void embedding(uintptr_t out, uintptr_t ids, uintptr_t table, int tokens, int hidden, int vocab,
               uintptr_t stream) {
  DLLM_HOST_CHECK(hidden % 8 == 0, "hidden % 8");
  if (tokens == 0) return;
  hipLaunchKernelGGL(embedding_kernel, dim3(tokens), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (bf16*)out, (const int32_t*)ids, (const bf16*)table, hidden, vocab);
  DLLM_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// K4 + K5: RoPE on q/k (rotate-half) fused with the paged KV-cache append.
// qkv [T, (Hq + 2 Hkv) * D] -> q_out [T, Hq, D] (rotated)
// k_cache [NB, Hkv, BS, D]; v_cache [NB, Hkv, D, BS] (transposed V).
// cos_sin [max_pos, D] f32 (first half cos, second half sin); nullptr = no RoPE (GPT-2).
// One workgroup per token; a thread owns 4 rotation pairs (8-byte vectors).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) rope_cache_kernel(bf16* __restrict__ q_out, const bf16* __restrict__ qkv,
                                                         const int32_t* __restrict__ positions,
                                                         const float* __restrict__ cos_sin,
                                                         bf16* __restrict__ k_cache, bf16* __restrict__ v_cache,
                                                         const int32_t* __restrict__ slots, int hq, int hkv,
                                                         int d, int bs, int do_v) {
  const int t = blockIdx.x;
  const int half = d >> 1;
  const int qpr = half >> 2;  // threads per head (4 pairs each)
  const int pos = positions[t];
  const int slot = slots[t];
  const int blk = slot / bs, off = slot % bs;
  const bf16* row = qkv + (size_t)t * (hq + 2 * hkv) * d;
  const float* cs = cos_sin ? cos_sin + (size_t)pos * d : nullptr;
  // q and k: rotate (q_out null: the attention kernel rotates q itself -- K / V only here)
  const int h0 = q_out ? 0 : hq;
  for (int i = threadIdx.x + h0 * qpr; i < (hq + hkv) * qpr; i += blockDim.x) {
    const int h = i / qpr, p = (i % qpr) * 4;
    const bf16* src = row + h * d;
    bf16x4 x1 = *reinterpret_cast<const bf16x4*>(src + p);
    bf16x4 x2 = *reinterpret_cast<const bf16x4*>(src + half + p);
    bf16x4 o1, o2;
    if (cs) {
      f32x4 c = *reinterpret_cast<const f32x4*>(cs + p);
      f32x4 s = *reinterpret_cast<const f32x4*>(cs + half + p);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float a = bf2f(x1[j]), b = bf2f(x2[j]);
        o1[j] = f2bf(a * c[j] - b * s[j]);
        o2[j] = f2bf(b * c[j] + a * s[j]);
      }
    } else {
      o1 = x1;
      o2 = x2;
    }
    bf16* dst;
    if (h < hq) {
      dst = q_out + ((size_t)t * hq + h) * d;
    } else {
      dst = k_cache + (((size_t)blk * hkv + (h - hq)) * bs + krow(off, bs)) * d;
    }
    *reinterpret_cast<bf16x4*>(dst + p) = o1;
    *reinterpret_cast<bf16x4*>(dst + half + p) = o2;
  }
  if (!do_v) return;  // v_group_kernel appends V
  // v: transposed store into [blk][h][d][bs]
  const bf16* vsrc = row + (hq + hkv) * d;
  for (int i = threadIdx.x; i < hkv * d; i += blockDim.x) {
    const int h = i / d, e = i % d;
    v_cache[((size_t)blk * hkv + h) * d * bs + vofs(off, e, d, bs)] = vsrc[i];
  }
}

// V append for a prefill batch, eight tokens per workgroup.  The transposed layouts keep a key's
// 8-aligned group of 8 contiguous per (head, e) -- vofs(off0 + j) = vofs(off0) + j when
// off0 % 8 == 0 and bs % 8 == 0 -- so when the group's slots are consecutive and 8-aligned (a
// prompt's tokens: consecutive slots from a block start) a thread writes one 16-byte vector where
// the per-token path scatters eight 2-byte stores (whole 64-byte lines instead of partial ones).
// Loads: for a fixed token j, a wave's 64 consecutive e read 128 contiguous bytes.  Any other group
// (a prompt boundary inside it, a sequence resuming mid-group, the batch tail) takes the per-token
// scatter.
__global__ void __launch_bounds__(256) v_group_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ v_cache,
                                                      const int32_t* __restrict__ slots, int tokens, int hq,
                                                      int hkv, int d, int bs) {
  __shared__ int sl[8];
  const int t0 = blockIdx.x * 8;
  const int n = min(8, tokens - t0);
  if (threadIdx.x < 8) sl[threadIdx.x] = threadIdx.x < n ? slots[t0 + threadIdx.x] : -1;
  __syncthreads();
  const int width = (hq + 2 * hkv) * d;
  const bf16* vsrc = qkv + (size_t)t0 * width + (hq + hkv) * d;
  bool full = n == 8 && sl[0] >= 0 && sl[0] % 8 == 0;
#pragma unroll
  for (int j = 1; j < 8; ++j) full = full && sl[j] == sl[0] + j;
  if (full) {
    const int blk = sl[0] / bs, off0 = sl[0] % bs;
    for (int i = threadIdx.x; i < hkv * d; i += blockDim.x) {
      const int h = i / d, e = i % d;
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = vsrc[(size_t)j * width + i];
      *reinterpret_cast<bf16x8*>(v_cache + ((size_t)blk * hkv + h) * d * bs + vofs(off0, e, d, bs)) = o;
    }
    return;
  }
  for (int j = 0; j < n; ++j) {
    const int blk = sl[j] / bs, off = sl[j] % bs;
    for (int i = threadIdx.x; i < hkv * d; i += blockDim.x) {
      const int h = i / d, e = i % d;
      v_cache[((size_t)blk * hkv + h) * d * bs + vofs(off, e, d, bs)] = vsrc[(size_t)j * width + i];
    }
  }
}

void rope_cache_append(uintptr_t q_out, uintptr_t qkv, uintptr_t positions, uintptr_t cos_sin,
                       uintptr_t k_cache, uintptr_t v_cache, uintptr_t slots, int tokens, int hq, int hkv,
                       int d, int bs, int v_groups, uintptr_t stream) {
  DLLM_HOST_CHECK(d % 8 == 0 && d <= 256, "head_dim must be a multiple of 8, <= 256");
  DLLM_HOST_CHECK(hq % hkv == 0, "Hq % Hkv");
  if (tokens == 0) return;
  const bool grouped = v_groups && bs % 8 == 0 && tokens >= 8;
  hipLaunchKernelGGL(rope_cache_kernel, dim3(tokens), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (bf16*)q_out, (const bf16*)qkv, (const int32_t*)positions, (const float*)cos_sin,
                     (bf16*)k_cache, (bf16*)v_cache, (const int32_t*)slots, hq, hkv, d, bs, grouped ? 0 : 1);
  DLLM_HIP_CHECK(hipGetLastError());
  if (!grouped) return;
  hipLaunchKernelGGL(v_group_kernel, dim3((tokens + 7) / 8), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const bf16*)qkv, (bf16*)v_cache, (const int32_t*)slots, tokens, hq, hkv, d, bs);
  DLLM_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// SwiGLU activation: gu [T, 2I] = [gate | up] -> out [T, I] = silu(gate) * up.
// Grid-stride over bf16x8 vectors.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) silu_mul_kernel(bf16* __restrict__ out, const bf16* __restrict__ gu,
                                                       int inter, long total_vec) {
  const int vpr = inter >> 3;
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < total_vec; v += (long)gridDim.x * 256) {
    const long t = v / vpr;
    const int c = (int)(v % vpr) * 8;
    bf16x8 g = *reinterpret_cast<const bf16x8*>(gu + t * 2 * inter + c);
    bf16x8 u = *reinterpret_cast<const bf16x8*>(gu + t * 2 * inter + inter + c);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(silu_f(bf2f(g[j])) * bf2f(u[j]));
    *reinterpret_cast<bf16x8*>(out + t * inter + c) = o;
  }
}

void silu_mul(uintptr_t out, uintptr_t gu, int tokens, int inter, uintptr_t stream) {
  DLLM_HOST_CHECK(inter % 8 == 0, "intermediate % 8");
  const long total = (long)tokens * (inter / 8);
  if (total == 0) return;
  long blocks = (total + 255) / 256;
  if (blocks > 256 * 8) blocks = 256 * 8;
  hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (bf16*)out, (const bf16*)gu, inter, total);
  DLLM_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// a <- a + b (bf16, 16-byte vectors): closes the residual stream at a stage boundary.
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) add_inplace_kernel(bf16* __restrict__ a, const bf16* __restrict__ b,
                                                          long nvec) {
  for (long v = (long)blockIdx.x * 256 + threadIdx.x; v < nvec; v += (long)gridDim.x * 256) {
    bf16x8 x = reinterpret_cast<bf16x8*>(a)[v];
    const bf16x8 y = reinterpret_cast<const bf16x8*>(b)[v];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = f2bf(bf2f(x[j]) + bf2f(y[j]));
    reinterpret_cast<bf16x8*>(a)[v] = x;
  }
}

void add_inplace(uintptr_t a, uintptr_t b, long n, uintptr_t stream) {
  DLLM_HOST_CHECK(n % 8 == 0, "numel % 8");
  const long nvec = n / 8;
  if (nvec == 0) return;
  long blocks = (nvec + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(add_inplace_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (bf16*)a, (const bf16*)b, nvec);
  DLLM_HIP_CHECK(hipGetLastError());
}

// ---------------------------------------------------------------------------
// K10 tail: greedy argmax over the vocabulary. One 1024-thread workgroup per row.
// Ties resolve to the smallest index (matches torch.argmax on the fp32 values).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void argmax_merge(float& bv, int& bi, float v, int i) {
  if (v > bv || (v == bv && i < bi) || (bv != bv)) { bv = v; bi = i; }
}

__global__ void __launch_bounds__(1024) argmax_kernel(int32_t* __restrict__ out, const bf16* __restrict__ logits,
                                                      int vocab, long row_stride) {
  __shared__ float sv[16];
  __shared__ int si[16];
  const bf16* row = logits + (size_t)blockIdx.x * row_stride;
  float bv = -INFINITY;
  int bi = 0x7fffffff;
  const int nvec = ((((uintptr_t)row) & 15) == 0) ? vocab >> 3 : 0;
  const bf16x8* rv = reinterpret_cast<const bf16x8*>(row);
  // four 16-byte loads in flight per thread before the first compare (one per iteration left the
  // 250 KB row at ~3.5 TB/s).  A thread visits its indices in increasing order, so inside its scan
  // a strict > keeps the smallest index among equal values (one compare and two selects, not the
  // cross-thread merge's tie and NaN rules)
  for (int v0 = threadIdx.x; v0 < nvec; v0 += 4 * 1024) {
    bf16x8 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = v0 + u * 1024;
      if (v < nvec) x[u] = rv[v];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int v = v0 + u * 1024;
      if (v < nvec) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xv = bf2f(x[u][j]);
          const bool take = xv > bv;
          bv = take ? xv : bv;
          bi = take ? v * 8 + j : bi;
        }
      }
    }
  }
  for (int i = nvec * 8 + threadIdx.x; i < vocab; i += 1024) argmax_merge(bv, bi, bf2f(row[i]), i);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float ov = __shfl_xor(bv, o, 64);
    int oi = __shfl_xor(bi, o, 64);
    argmax_merge(bv, bi, ov, oi);
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) { sv[wid] = bv; si[wid] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < 16; ++w) argmax_merge(bv, bi, sv[w], si[w]);
    out[blockIdx.x] = bi;
  }
}

void argmax(uintptr_t out, uintptr_t logits, int rows, int vocab, long row_stride, uintptr_t stream) {
  if (rows == 0) return;
  hipLaunchKernelGGL(argmax_kernel, dim3(rows), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream),
                     (int32_t*)out, (const bf16*)logits, vocab, row_stride);
  DLLM_HIP_CHECK(hipGetLastError());
}

}  // namespace dllm
