// K11 + K12: Mixtral mixture-of-experts on gfx950, graph-capturable (no host round trip).
//
//  moe_route    : router logits [T,E] -> softmax -> top-k -> renormalise (Mixtral); per-expert
//                 counts, offsets and the expert-sorted assignment list (slot -> token) plus the
//                 inverse map ((t,j) -> slot), in ONE 1024-thread workgroup (LDS counters + scan).
//  moe_grouped  : per-expert weight-streaming GEMM (grid = column tiles x experts), A rows
//                 gathered through the sorted list, rows processed in 64-row chunks; epilogue
//                 SwiGLU (gate|up experts weight [E, 2I, H]) or plain store (down [E, H, I]).
//                 Every expert's weights stream once per chunk; the decode regime has <= 64 rows
//                 per expert, i.e. one pass.
//  moe_combine  : out[t] = sum_j w[t,j] * y[inv[t,j]]   (fixed j order: deterministic)
#include "skinny_common.h"
#include "launchers.h"

namespace dllm {

constexpr int kMaxExperts = 64;

__global__ void __launch_bounds__(1024) moe_route_kernel(const bf16* __restrict__ logits, int T, int E, int k,
                                                         float* __restrict__ topk_w, int* __restrict__ topk_ids,
                                                         int* __restrict__ counts, int* __restrict__ offsets,
                                                         int* __restrict__ sorted_tok, int* __restrict__ inv) {
  __shared__ int cnt[kMaxExperts], cur[kMaxExperts];
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    float p[kMaxExperts];
    float mx = -INFINITY;
    for (int e = 0; e < E; ++e) {
      p[e] = bf2f(logits[(size_t)t * E + e]);
      mx = fmaxf(mx, p[e]);
    }
    float s = 0.f;
    for (int e = 0; e < E; ++e) {
      p[e] = __expf(p[e] - mx);
      s += p[e];
    }
    float tot = 0.f;
    int ids[8];
    float ws[8];
    for (int j = 0; j < k; ++j) {
      int best = 0;
      float bv = -1.f;
      for (int e = 0; e < E; ++e)
        if (p[e] > bv) { bv = p[e]; best = e; }
      ids[j] = best;
      ws[j] = bv / s;
      tot += ws[j];
      p[best] = -2.f;
    }
    for (int j = 0; j < k; ++j) {
      topk_ids[t * k + j] = ids[j];
      topk_w[t * k + j] = ws[j] / tot;
      atomicAdd(&cnt[ids[j]], 1);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int acc = 0;
    for (int e = 0; e < E; ++e) {
      offsets[e] = acc;
      cur[e] = acc;
      counts[e] = cnt[e];
      acc += cnt[e];
    }
    offsets[E] = acc;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < T; t += blockDim.x) {
    for (int j = 0; j < k; ++j) {
      const int e = topk_ids[t * k + j];
      const int slot = atomicAdd(&cur[e], 1);
      sorted_tok[slot] = t;
      inv[t * k + j] = slot;
    }
  }
}

constexpr int MOE_EPI_STORE = 0;
constexpr int MOE_EPI_SWIGLU = 1;

// y[slot, :] for the rows of expert blockIdx.y.  x rows: gather ? x[gather[slot]] : x[slot].
template <int NT, int EPI>
__global__ void __launch_bounds__(512, 1) moe_grouped_kernel(bf16* __restrict__ y, const bf16* __restrict__ x,
                                                             const int* __restrict__ gather,
                                                             const bf16* __restrict__ w, const int* __restrict__ counts,
                                                             const int* __restrict__ offsets, int N, int K, int ldy) {
  constexpr int MT = 4, BM = 64, BN = NT * 16;
  __shared__ __attribute__((aligned(16))) float red[BM * BN];
  const int e = blockIdx.y;
  const int cnt = counts[e];
  if (cnt == 0) return;                       // uniform across the workgroup
  const int off = offsets[e];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int r = lane & 15, g = lane >> 4;
  const bf16* we = w + (size_t)e * N * K;
  const bf16* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    int n0;
    if (EPI == MOE_EPI_SWIGLU) n0 = (nt < NT / 2 ? 0 : N / 2) + blockIdx.x * (BN / 2) + (nt % (NT / 2)) * 16;
    else n0 = blockIdx.x * BN + nt * 16;
    wrow[nt] = we + (size_t)(n0 + r) * K + 32 * g;
  }
  const int ngroups = K >> 7;
  const int per = (ngroups + kSkWaves - 1) / kSkWaves;
  const int g0 = wv * per, g1 = min(ngroups, g0 + per);
  for (int r0 = 0; r0 < cnt; r0 += BM) {
    const int rows = min(BM, cnt - r0);
    for (int i = threadIdx.x; i < BM * BN; i += 512) red[i] = 0.f;
    const bf16* xrow[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int slot = off + r0 + min(mt * 16 + r, rows - 1);
      const int src = gather ? gather[slot] : slot;
      xrow[mt] = x + (size_t)src * K + 32 * g;
    }
    f32x4 acc[MT][NT];
    sk_mainloop<MT, NT>(acc, xrow, wrow, g0, g1);
    __syncthreads();
    sk_reduce_lds<MT, NT>(red, acc, lane);
    __syncthreads();
    if (EPI == MOE_EPI_SWIGLU) {
      constexpr int HB = BN / 2;
      for (int q = threadIdx.x; q < rows * HB; q += 512) {
        const int m = q / HB, c = q % HB;
        y[(size_t)(off + r0 + m) * ldy + blockIdx.x * HB + c] = f2bf(silu_f(red[m * BN + c]) * red[m * BN + HB + c]);
      }
    } else {
      for (int q = threadIdx.x; q < rows * BN; q += 512) {
        const int m = q / BN, c = q % BN;
        y[(size_t)(off + r0 + m) * ldy + blockIdx.x * BN + c] = f2bf(red[m * BN + c]);
      }
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) moe_combine_kernel(bf16* __restrict__ out, const bf16* __restrict__ ysorted,
                                                          const float* __restrict__ topk_w,
                                                          const int* __restrict__ inv, int H, int k) {
  const int t = blockIdx.x;
  for (int v = threadIdx.x; v < (H >> 3); v += 256) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < k; ++j) {
      const float wj = topk_w[t * k + j];
      const bf16x8 yv = *reinterpret_cast<const bf16x8*>(ysorted + (size_t)inv[t * k + j] * H + v * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += wj * bf2f(yv[i]);
    }
    bf16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = f2bf(acc[i]);
    *reinterpret_cast<bf16x8*>(out + (size_t)t * H + v * 8) = o;
  }
}

// ------------------------------------------------------------------ launchers
void moe_route(uintptr_t logits, int T, int E, int k, uintptr_t topk_w, uintptr_t topk_ids, uintptr_t counts,
               uintptr_t offsets, uintptr_t sorted_tok, uintptr_t inv, uintptr_t stream) {
  DLLM_HOST_CHECK(E >= 1 && E <= kMaxExperts, "1 <= experts <= 64");
  DLLM_HOST_CHECK(k >= 1 && k <= 8 && k <= E, "1 <= top_k <= min(8, experts)");
  hipLaunchKernelGGL(moe_route_kernel, dim3(1), dim3(1024), 0, reinterpret_cast<hipStream_t>(stream),
                     (const bf16*)logits, T, E, k, (float*)topk_w, (int*)topk_ids, (int*)counts, (int*)offsets,
                     (int*)sorted_tok, (int*)inv);
  DLLM_HIP_CHECK(hipGetLastError());
}

// mode 1 (SwiGLU): w [E, 2I, K] -> y [T*k, I]; mode 0: w [E, N, K] -> y [T*k, N]
void moe_grouped_gemm(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                      int E, int N, int K, int mode, uintptr_t stream) {
  DLLM_HOST_CHECK(K % 128 == 0, "K % 128");
  DLLM_HOST_CHECK(N % 32 == 0, "N % 32");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (mode == 1) {
    hipLaunchKernelGGL((moe_grouped_kernel<2, MOE_EPI_SWIGLU>), dim3(N / 2 / 16, E), dim3(512), 0, s, (bf16*)y,
                       (const bf16*)x, (const int*)gather, (const bf16*)w, (const int*)counts,
                       (const int*)offsets, N, K, N / 2);
  } else {
    hipLaunchKernelGGL((moe_grouped_kernel<2, MOE_EPI_STORE>), dim3(N / 32, E), dim3(512), 0, s, (bf16*)y,
                       (const bf16*)x, (const int*)gather, (const bf16*)w, (const int*)counts,
                       (const int*)offsets, N, K, N);
  }
  DLLM_HIP_CHECK(hipGetLastError());
}

void moe_combine(uintptr_t out, uintptr_t ysorted, uintptr_t topk_w, uintptr_t inv, int T, int H, int k,
                 uintptr_t stream) {
  DLLM_HOST_CHECK(H % 8 == 0, "H % 8");
  if (T == 0) return;
  hipLaunchKernelGGL(moe_combine_kernel, dim3(T), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), (bf16*)out,
                     (const bf16*)ysorted, (const float*)topk_w, (const int*)inv, H, k);
  DLLM_HIP_CHECK(hipGetLastError());
}

}  // namespace dllm
