// Large-batch decode GEMM (M = 64..512): C[M,N] = A[M,K] . B[N,K]^T, bf16 in, f32 accumulate.
//
// Why: at these M hipBLASLt's tiles leave most of the 256 CUs idle for N <= 6144
// (qkv / o / down run at 1.1-2 TB/s and 0.3-0.5 PF, bench/blas_graph_probe.py).  This kernel
// splits K across workgroups so (N/128) x (M/128) x S fills the chip, and reduces the S f32
// partial slabs in a second, fully parallel pass (optionally with the SwiGLU epilogue).
//
// Structure (the guide's minimum 2-phase LDS pipeline, gfx950):
//  * tile 128 x 128 x 64, 256 threads = 4 waves in 2 x 2, wave tile 64 x 64 = 4 x 4
//    v_mfma_f32_16x16x32_bf16 accumulators (64 VGPRs);
//  * global -> LDS with global_load_lds_dwordx4 (16 B per lane, lane-linear 1 KiB per
//    wave-instruction = 8 rows x 128 B); the bank-conflict swizzle (16-B chunk c of row r
//    stored at c ^ ((r >> 1) & 7)) is applied on the per-lane SOURCE address and on the
//    ds_read address (guide rule 21), which makes the 16-lane ds_read_b128 groups
//    conflict-free;
//  * double-buffered LDS (64 KiB): stage tile t+1 before the MFMAs of tile t, one
//    vmcnt(0) + barrier per K-tile.
#include "common.h"
#include "launchers.h"

#include <cstdlib>

namespace dllm {

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;

constexpr int TBM = 128, TBN = 128, TBK = 64;
constexpr int TILE_ELEMS = TBM * TBK;   // 8192 bf16 = 16 KiB

__device__ __forceinline__ int swz_chunk(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <bool SPLIT>
__global__ void __launch_bounds__(256, 2) gemm_tiled_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                            bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                            int K, int k_per_split) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * 2 * TILE_ELEMS];   // [buf][A|B][128][64]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wm = wv >> 1, wn = wv & 1;
  // 1-D grid, XCD-aware: hardware dispatches block b to XCD b % 8, so logical tile
  // (b % 8) * (total / 8) + b / 8 gives each XCD a contiguous run of logical ids; M is the
  // fastest logical axis, so the M tiles that share a W tile run back-to-back on ONE XCD and
  // the second reads W from that XCD's L2 instead of HBM.
  const int mtiles = (M + TBM - 1) / TBM, total = gridDim.x;
  int b = blockIdx.x;
  if ((total & 7) == 0) b = (b & 7) * (total >> 3) + (b >> 3);
  const int m_t = b % mtiles, rest = b / mtiles;
  const int nsplit = total / (mtiles * (N / TBN));
  const int split = rest % nsplit, n_t = rest / nsplit;
  const int n0 = n_t * TBN, m0 = m_t * TBM;
  const int kb = split * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int nt = max(0, (ke - kb) / TBK);

  // staging addresses (per lane): instruction i = wv*4 + j covers tile rows 8i .. 8i+7
  const bf16* srcA[4];
  const bf16* srcB[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = wv * 4 + j;
    const int r = 8 * i + (lane >> 3);
    const int c = swz_chunk(r, lane & 7);
    srcA[j] = A + (size_t)min(m0 + r, M - 1) * K + c * 8;
    srcB[j] = B + (size_t)(n0 + r) * K + c * 8;
  }
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = wv * 4 + j;
      __builtin_amdgcn_global_load_lds((glb_vptr)(srcA[j] + k0), (lds_vptr)(smem + (buf * 2 + 0) * TILE_ELEMS + i * 512),
                                       16, 0, 0);
      __builtin_amdgcn_global_load_lds((glb_vptr)(srcB[j] + k0), (lds_vptr)(smem + (buf * 2 + 1) * TILE_ELEMS + i * 512),
                                       16, 0, 0);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  if (nt > 0) {
    stage(0, kb);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int t = 0; t < nt; ++t) {
      const int cur = t & 1;
      if (t + 1 < nt) stage(cur ^ 1, kb + (t + 1) * TBK);
      const bf16* sa = smem + (cur * 2 + 0) * TILE_ELEMS;
      const bf16* sb = smem + (cur * 2 + 1) * TILE_ELEMS;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 fa[4], fb[4];
#pragma unroll
        for (int rt = 0; rt < 4; ++rt) {
          const int row = wm * 64 + rt * 16 + fr;
          fa[rt] = *reinterpret_cast<const bf16x8*>(sa + row * TBK + swz_chunk(row, 4 * s + fq) * 8);
        }
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const int row = wn * 64 + ct * 16 + fr;
          fb[ct] = *reinterpret_cast<const bf16x8*>(sb + row * TBK + swz_chunk(row, 4 * s + fq) * 8);
        }
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
#pragma unroll
          for (int ct = 0; ct < 4; ++ct)
            acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rt], fb[ct], acc[rt][ct], 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  }
  // epilogue: lane holds col (lane&15), rows 4*(lane>>4)+i of each 16x16 tile
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + rt * 16 + 4 * fq + i;
      if (m >= M) continue;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int n = n0 + wn * 64 + ct * 16 + fr;
        if (SPLIT) part_store(P, ((size_t)split * M + m) * N + n, acc[rt][ct][i]);
        else C[(size_t)m * N + n] = f2bf(acc[rt][ct][i]);
      }
    }
  }
}

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
  // DLLM_SKN_THREADS=512: 512-thread workgroups (8 waves per row, one vector per thread at hidden
  // 4096); the sum of squares is then reduced over 8 wave partials, so the output is no longer
  // bit-identical to splitk_reduce + rms_norm_kernel (A/B knob, profiles/wide_gemm.md).  Only
  // instantiated for S == 8 slabs and 2048 < hidden <= 4096 (256 < N/8 <= 512); every other shape
  // keeps the 256-thread kernel.  Read once per process (first call).
  // tests/test_gemm_gpu.py::test_skn_512_threads covers it in a subprocess.
  static const int nth = [] {
    const char* e = getenv("DLLM_SKN_THREADS");
    return e && atoi(e) == 512 ? 512 : 256;
  }();
  const int nvec = N / 8;
  const int bth = (nth == 512 && nvec > 256 && nvec <= 512 && S == 8) ? 512 : 256;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(M), dim3(bth), 0, s, (bf16*)y, (bf16*)residual, (const float*)ws, S, M, N,
                       (const bf16*)w, eps, (uint8_t*)q8, (float*)qs);
  };
  if (bth == 512) {
    go(splitk_add_rms_norm_kernel<1, 8, 512>);
    DLLM_HIP_CHECK(hipGetLastError());
    return;
  }
  static const bool const_slabs = [] {
    const char* e = getenv("DLLM_SKN_CONST");
    return !(e && e[0] == '0');
  }();
#define DLLM_SKN(MV)                                                   \
  do {                                                                 \
    if (!const_slabs) go(splitk_add_rms_norm_kernel<MV, 0>);           \
    else if (S == 8) go(splitk_add_rms_norm_kernel<MV, 8>);                 \
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

// plain split-K reduce of partials left by gemm_tiled(mode 2): out = bf16(sum_s P[s]) (+bias)
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

// mode 0: C[M,N] = A B^T (+bias);  mode 1 (SwiGLU): C[M, N/2] = silu(A Bg^T) * (A Bu^T), B = [Bg; Bu]
void gemm_tiled(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t bias, uintptr_t ws, long ws_floats, int M, int N,
                int K, int splits, int mode, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(N % TBN == 0, "N must be a multiple of 128");
  DLLM_HOST_CHECK(K % TBK == 0, "K must be a multiple of 64");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");   // 2: leave partial slabs in ws, no reduce
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int kps = (K / TBK + splits - 1) / splits * TBK;
  const int S = (K + kps - 1) / kps;
  dim3 grid((N / TBN) * ((M + TBM - 1) / TBM) * S);
  DLLM_HOST_CHECK(mode != 2 || S > 1, "mode 2 needs a K split");
  if (S == 1 && mode == 0 && bias == 0) {
    hipLaunchKernelGGL(gemm_tiled_kernel<false>, grid, dim3(256), 0, s, (const bf16*)a, (const bf16*)b, (bf16*)c,
                       (float*)nullptr, M, N, K, kps);
    DLLM_HIP_CHECK(hipGetLastError());
    return;
  }
  DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  hipLaunchKernelGGL(gemm_tiled_kernel<true>, grid, dim3(256), 0, s, (const bf16*)a, (const bf16*)b, (bf16*)nullptr,
                     (float*)ws, M, N, K, kps);
  DLLM_HIP_CHECK(hipGetLastError());
  if (mode == 2) return;
  splitk_reduce_ex(c, ws, bias, S, M, N, mode == 1, stream);
}

}  // namespace dllm
