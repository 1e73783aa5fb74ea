// Issue cost of a wave's staging instructions on gfx950: N back-to-back global_load_lds_dwordx4
// (LDS-DMA, 1 KiB per wave-instruction) vs global_load_dwordx4 into VGPRs, every CU busy (4 waves
// per CU, one per SIMD), timed with s_memtime around the issue run (issue only: no wait) and
// around issue + vmcnt(0).  Sources stream a 1 GiB buffer (HBM) in 128-byte rows, 8 rows per
// wave-instruction (the GEMM staging shape).  hipcc --offload-arch=gfx950 -O3 issue_cost.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

typedef __attribute__((address_space(3))) void* lds_p;
typedef __attribute__((address_space(1))) void* glb_p;
typedef int int4v __attribute__((ext_vector_type(4)));

constexpr int N = 12;                 // instructions per run (one K-tile of the BN = 128 GEMM)
constexpr int REPS = 64;

template <int MODE>   // 0: LDS-DMA, 1: global_load_dwordx4 -> VGPR
__global__ void __launch_bounds__(256, 1) k(const char* __restrict__ src, long span, unsigned long long* out,
                                            int* sink) {
  __shared__ __attribute__((aligned(16))) char lds[4 * N * 1024];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long row_bytes = 8192;                      // K = 4096 bf16 rows
  unsigned long long t_issue = 0, t_all = 0;
  int4v acc = {0, 0, 0, 0};
  long base = ((long)blockIdx.x * 4 + wv) * (N * 8 * row_bytes);
  for (int r = 0; r < REPS; ++r) {
    const long off = (base + (long)r * 128 + (long)(lane >> 3) * row_bytes + (lane & 7) * 16) % (span - (long)N * 8 * row_bytes);
    unsigned long long t0, t1, t2;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < N; ++i)
        __builtin_amdgcn_global_load_lds((glb_p)(src + off + (long)i * 8 * row_bytes), (lds_p)(lds + (wv * N + i) * 1024),
                                         16, 0, 0);
    } else {
      int4v v[N];
#pragma unroll
      for (int i = 0; i < N; ++i) v[i] = *reinterpret_cast<const int4v*>(src + off + (long)i * 8 * row_bytes);
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < N; ++i) acc += v[i];
    }
    if constexpr (MODE == 0) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t2)::"memory");
    if (r >= 4) { t_issue += t1 - t0; t_all += t2 - t0; }
  }
  if (lane == 0) {
    out[(blockIdx.x * 4 + wv) * 2] = t_issue;
    out[(blockIdx.x * 4 + wv) * 2 + 1] = t_all;
  }
  if (acc[0] == 12345) sink[0] = acc[1] + lds[lane];
}

int main() {
  const long span = 1L << 30;
  char* src;
  unsigned long long* out;
  int* sink;
  hipMalloc(&src, span);
  hipMemset(src, 1, span);
  hipMalloc(&out, 256 * 4 * 2 * sizeof(unsigned long long));
  hipMalloc(&sink, 64);
  for (int mode = 0; mode < 2; ++mode) {
    for (int it = 0; it < 3; ++it) {
      if (mode == 0) hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, src, span, out, sink);
      else hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, src, span, out, sink);
      hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(256 * 4 * 2);
    hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<double> iss, all;
    for (int w = 0; w < 256 * 4; ++w) {
      iss.push_back(h[2 * w] / double(REPS - 4) / N);
      all.push_back(h[2 * w + 1] / double(REPS - 4));
    }
    std::sort(iss.begin(), iss.end());
    std::sort(all.begin(), all.end());
    printf("%s: issue cycles per instruction median %.1f (p10 %.1f p90 %.1f); %d instructions issue+land median %.0f cycles\n",
           mode == 0 ? "global_load_lds_dwordx4" : "global_load_dwordx4   ", iss[iss.size() / 2], iss[iss.size() / 10],
           iss[9 * iss.size() / 10], N, all[all.size() / 2]);
  }
  return 0;
}
