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

// Router GEMV + top-k fused (decode): one wave per token computes its E router logits
// (H split over the 64 lanes, 16-B loads, wave reductions), rounds them to bf16 like the
// library-GEMM path it replaces, then lane 0 applies softmax -> top-k -> renormalise.
// moe_scatter_kernel (one workgroup) then counts per expert in LDS, scans, and writes the
// offsets and the expert-sorted slot lists (no global counters: nothing to zero first, so the
// pair stays a plain two-node piece of a captured graph).  Replaces linear(x, W_router) + the single-workgroup moe_route_kernel
// (14 + 11 us per layer at T = 256).
template <int E>
__global__ void __launch_bounds__(256) moe_router_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w, int T,
                                                         int H, int k, float* __restrict__ topk_w,
                                                         int* __restrict__ topk_ids) {
  // one workgroup per token, the 4 waves split H (a wave per token left 3/4 of the CUs idle at
  // T = 256 and walked 8 dependent load rounds: 10.5 us per Mixtral layer)
  __shared__ float part[4][E];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int t = blockIdx.x;
  float acc[E];
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = 0.f;
  const bf16* xr = x + (size_t)t * H;
  const int hq = H / 4;
  for (int c = wv * hq + lane * 8; c < (wv + 1) * hq; c += 64 * 8) {
    const bf16x8 xv = *reinterpret_cast<const bf16x8*>(xr + c);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const bf16x8 wt = *reinterpret_cast<const bf16x8*>(w + (size_t)e * H + c);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[e] += bf2f(xv[i]) * bf2f(wt[i]);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) acc[e] = wave_sum(acc[e]);
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < E; ++e) part[wv][e] = acc[e];
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  float p[E];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    p[e] = bf2f(f2bf(((part[0][e] + part[1][e]) + part[2][e]) + part[3][e]));
    mx = fmaxf(mx, p[e]);
  }
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    p[e] = __expf(p[e] - mx);
    sum += p[e];
  }
  int ids[8];
  float ws[8];
  float tot = 0.f;
  for (int j = 0; j < k; ++j) {
    int best = 0;
    float bv = -1.f;
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (p[e] > bv) { bv = p[e]; best = e; }
    ids[j] = best;
    ws[j] = bv / sum;
    tot += ws[j];
    p[best] = -2.f;
  }
  for (int j = 0; j < k; ++j) {
    topk_ids[t * k + j] = ids[j];
    topk_w[t * k + j] = ws[j] / tot;
  }
}

__global__ void __launch_bounds__(1024) moe_scatter_kernel(const int* __restrict__ topk_ids, int T, int E, int k,
                                                           int* __restrict__ counts, int* __restrict__ offsets,
                                                           int* __restrict__ sorted_tok, int* __restrict__ inv) {
  __shared__ int cnt[kMaxExperts], cur[kMaxExperts];
  for (int e = threadIdx.x; e < E; e += blockDim.x) cnt[e] = 0;
  __syncthreads();
  for (int i = threadIdx.x; i < T * k; i += blockDim.x) atomicAdd(&cnt[topk_ids[i]], 1);
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
  for (int i = threadIdx.x; i < T * k; i += blockDim.x) {
    const int slot = atomicAdd(&cur[topk_ids[i]], 1);
    sorted_tok[slot] = i / k;
    inv[i] = slot;
  }
}

constexpr int MOE_EPI_STORE = 0;
constexpr int MOE_EPI_SWIGLU = 1;

// Rows [0, cnt) of one expert in chunks of MT*16 rows; every chunk streams the WG's W column
// tile once (K split over the WAVES waves, partial tiles summed through LDS).
template <int MT, int NT, int WAVES, int EPI>
__device__ __forceinline__ void moe_rows(float* red, bf16* __restrict__ y, const bf16* __restrict__ x,
                                         const int* __restrict__ gather, const bf16* const (&wrow)[NT], int cnt,
                                         int off, int K, int ldy, int g0, int g1, int lane) {
  constexpr int BM = MT * 16, BN = NT * 16, NTHR = WAVES * 64;
  const int r = lane & 15, g = lane >> 4;
  for (int r0 = 0; r0 < cnt; r0 += BM) {
    const int rows = min(BM, cnt - r0);
    for (int i = threadIdx.x; i < BM * BN; i += NTHR) red[i] = 0.f;
    const bf16* xrow[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int slot = off + r0 + min(mt * 16 + r, rows - 1);
      const int src = gather ? gather[slot] : slot;
      xrow[mt] = x + (size_t)src * K + 8 * g;
    }
    f32x4 acc[MT][NT];
    sk_mainloop<MT, NT>(acc, xrow, wrow, g0, g1);
    __syncthreads();
    sk_reduce_lds<MT, NT, WAVES>(red, acc, lane, threadIdx.x >> 6);
    if (EPI == MOE_EPI_SWIGLU) {
      constexpr int HB = BN / 2;
      for (int q = threadIdx.x; q < rows * HB; q += NTHR) {
        const int m = q / HB, c = q % HB;
        y[(size_t)(off + r0 + m) * ldy + blockIdx.x * HB + c] = f2bf(silu_f(red[m * BN + c]) * red[m * BN + HB + c]);
      }
    } else {
      for (int q = threadIdx.x; q < rows * BN; q += NTHR) {
        const int m = q / BN, c = q % BN;
        y[(size_t)(off + r0 + m) * ldy + blockIdx.x * BN + c] = f2bf(red[m * BN + c]);
      }
    }
    __syncthreads();
  }
}

// Grouped expert GEMM: grid (N / (NT*16), E).  The row tile is chosen PER EXPERT from its
// actual count (a workgroup-uniform branch): 16-row tiles for <= 16 rows, 32 for <= 32, else
// MTMAX*16-row chunks -- so routing imbalance never makes an expert re-stream its weights
// while it fits one chunk, and a decode expert with 10 rows does not gather 64.
template <int MTMAX, int NT, int WAVES, int EPI>
__global__ void __launch_bounds__(WAVES * 64, 1) moe_grouped_kernel(bf16* __restrict__ y, const bf16* __restrict__ x,
                                                                    const int* __restrict__ gather,
                                                                    const bf16* __restrict__ w,
                                                                    const int* __restrict__ counts,
                                                                    const int* __restrict__ offsets, int N, int K,
                                                                    int ldy) {
  constexpr int BN = NT * 16;
  __shared__ __attribute__((aligned(16))) float red[MTMAX * 16 * BN];
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
    wrow[nt] = we + (size_t)(n0 + r) * K + 8 * g;
  }
  const int ngroups = K >> 7;
  const int per = (ngroups + WAVES - 1) / WAVES;
  const int g0 = wv * per, g1 = min(ngroups, g0 + per);
  if (MTMAX == 1 || cnt <= 16) {
    moe_rows<1, NT, WAVES, EPI>(red, y, x, gather, wrow, cnt, off, K, ldy, g0, g1, lane);
  } else if constexpr (MTMAX >= 2) {
    if (MTMAX == 2 || cnt <= 32) moe_rows<2, NT, WAVES, EPI>(red, y, x, gather, wrow, cnt, off, K, ldy, g0, g1, lane);
    else if constexpr (MTMAX >= 4) moe_rows<4, NT, WAVES, EPI>(red, y, x, gather, wrow, cnt, off, K, ldy, g0, g1, lane);
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

// router GEMV + top-k + scatter (decode): x [T, H], w_router [E, H]
void moe_router_route(uintptr_t x, uintptr_t w, int T, int H, int E, int k, uintptr_t topk_w, uintptr_t topk_ids,
                      uintptr_t counts, uintptr_t offsets, uintptr_t sorted_tok, uintptr_t inv, uintptr_t stream) {
  DLLM_HOST_CHECK(E == 8 || E == 16, "fused router: 8 or 16 experts");
  DLLM_HOST_CHECK(k >= 1 && k <= 8 && k <= E, "1 <= top_k <= min(8, experts)");
  DLLM_HOST_CHECK(H % 8 == 0, "H % 8");
  if (T == 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  DLLM_HOST_CHECK(H % 32 == 0, "router: H % 32 (4 waves x 8-element vectors)");
  const dim3 grid(T);
  if (E == 8)
    hipLaunchKernelGGL(moe_router_kernel<8>, grid, dim3(256), 0, s, (const bf16*)x, (const bf16*)w, T, H, k,
                       (float*)topk_w, (int*)topk_ids);
  else
    hipLaunchKernelGGL(moe_router_kernel<16>, grid, dim3(256), 0, s, (const bf16*)x, (const bf16*)w, T, H, k,
                       (float*)topk_w, (int*)topk_ids);
  DLLM_HIP_CHECK(hipGetLastError());
  hipLaunchKernelGGL(moe_scatter_kernel, dim3(1), dim3(1024), 0, s, (const int*)topk_ids, T, E, k, (int*)counts,
                     (int*)offsets, (int*)sorted_tok, (int*)inv);
  DLLM_HIP_CHECK(hipGetLastError());
}

template <int MTMAX, int NT, int WAVES>
static void launch_grouped(hipStream_t s, bf16* y, const bf16* x, const int* gather, const bf16* w, const int* counts,
                           const int* offsets, int E, int N, int K, int mode) {
  constexpr int BN = NT * 16;
  if (mode == 1) {
    DLLM_HOST_CHECK(N % BN == 0, "moe grouped: 2I must be a multiple of the column tile");
    hipLaunchKernelGGL((moe_grouped_kernel<MTMAX, NT, WAVES, MOE_EPI_SWIGLU>), dim3(N / BN, E), dim3(WAVES * 64), 0,
                       s, y, x, gather, w, counts, offsets, N, K, N / 2);
  } else {
    DLLM_HOST_CHECK(N % BN == 0, "moe grouped: N must be a multiple of the column tile");
    hipLaunchKernelGGL((moe_grouped_kernel<MTMAX, NT, WAVES, MOE_EPI_STORE>), dim3(N / BN, E), dim3(WAVES * 64), 0, s,
                       y, x, gather, w, counts, offsets, N, K, N);
  }
}

// mode 1 (SwiGLU): w [E, 2I, K] -> y [T*k, I]; mode 0: w [E, N, K] -> y [T*k, N].
// rows_hint = expected rows per expert (T*k/E) picks the kernel family; variant > 0 forces one
// (benchmarking: 1 = <1,4,8>, 2 = <2,4,8>, 3 = <4,2,8>, 4 = <2,4,4>, 5 = <4,4,4>, 6 = <2,2,8>).
void moe_grouped_gemm(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets,
                      int E, int N, int K, int mode, int rows_hint, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(K % 128 == 0, "K % 128");
  DLLM_HOST_CHECK(N % 64 == 0, "N % 64");   // every column tile (32 or 64) divides N
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  auto args = [&](auto f) {
    f(s, (bf16*)y, (const bf16*)x, (const int*)gather, (const bf16*)w, (const int*)counts, (const int*)offsets, E, N,
      K, mode);
  };
  // measured (bench/moe_bench.py, Mixtral shapes): 4-wave <4,4,4> is best or tied at every
  // decode token count -- 4.4 TB/s at T=16, 3.8 at T=64, 3.0 at T=128 -- the 8-wave forms
  // spill and split K too finely (profiles/moe_grouped_variants.txt)
  (void)rows_hint;
  if (variant <= 0) variant = 5;
  switch (variant) {
    case 1: args(launch_grouped<1, 4, 8>); break;
    case 2: args(launch_grouped<2, 4, 8>); break;
    case 3: args(launch_grouped<4, 2, 8>); break;
    case 4: args(launch_grouped<2, 4, 4>); break;
    case 5: args(launch_grouped<4, 4, 4>); break;
    case 6: args(launch_grouped<2, 2, 8>); break;
    default: DLLM_HOST_CHECK(false, "moe grouped: unknown variant");
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
