// Ping-pong MFMA GEMM for 256-row tiles: C[M,N] = A[M,K] . B[N,K]^T, bf16 in, f32 accumulate.
// Serves the decode projections at batch 129..256 (one row tile, split-K over workgroups) and the
// prefill projections (M = tokens, grouped row-tile order, SwiGLU fused into the epilogue).
//
// Why (profiles/round3_decode_gemms.md): the 256 x 128 / 3-buffer kernel (gemm_wide.hip) runs
// all 8 waves in lock step -- one barrier per 64-deep K-tile, every wave of a SIMD reading its
// fragments at the same moment -- so its MFMA phase alone reaches ~55 % of peak, and its split-K
// epilogue stores one 2-byte element per lane (4 x 32-byte segments per store instruction).
//
// Structure (gfx950, wave64, 512 threads = 8 waves):
//  * tile 256 x BN (BN = 256: waves 2 (M) x 4 (N), wave tile 128 x 64; BN = 128: 4 x 2, 64 x 64),
//    v_mfma_f32_16x16x32_bf16, 16 independent accumulators per phase;
//  * K advances in 32-deep K-steps held in an LDS ring of NS slots (BN 256: 5 x 32 KiB, BN 128:
//    6 x 24 KiB, 160 / 144 KiB): slot = A [256][64 B] + B [BN][64 B] filled by
//    global_load_lds_dwordx4 (1 KiB = 16 rows per wave-instruction), the 16-byte chunk swizzle
//    c ^ ((row >> 1) & 3) on the per-lane SOURCE address and on the fragment read (conflict-free
//    ds_read_b128 for the 16 x 16 x 32 operand pattern on 64-byte rows; rule 21);
//  * NS - 1 K-steps in flight (96 KiB per CU), COUNTED s_waitcnt vmcnt(N) once per K-step, raw
//    s_barrier (never __syncthreads, which would drain the LDS-DMA queue);
//  * ping-pong: each K-step is P = rows / 64 phases of {fragment reads + staging issue | barrier |
//    16 MFMAs | barrier}; waves 4-7 (one per SIMD) start one barrier late, so on every SIMD one
//    wave's fragment reads and LDS-DMA issue run beside its partner's MFMA burst
//    (MI355X_MICROARCH "Two waves per SIMD", cdna_hip_programming §5 8-phase template);
//  * operands swapped in the MFMA (B fragment first), so a lane's accumulator holds 4 CONSECUTIVE
//    output columns of one row: the epilogue packs them 8 bytes at a time into an LDS image of the
//    output tile (padded rows, conflict-free), then every lane stores 16-byte row chunks --
//    full 128-byte lines for bf16 outputs, f16 split-K slabs and the SwiGLU product alike;
//  * SwiGLU without a weight permutation: the B tile's 16-row groups alternate gate / up rows of
//    the fused [2I, K] weight, so gate and up of an output column meet in one lane.
#include "common.h"
#include "launchers.h"

namespace dllm {

namespace {
constexpr int PBK = 32;                       // K per ring slot (64-byte rows)
typedef __attribute__((address_space(3))) void* lds_vptr_p;
typedef __attribute__((address_space(1))) void* glb_vptr_p;

__device__ __forceinline__ int pswz(int row, int chunk) { return chunk ^ ((row >> 1) & 3); }

template <int OFF>
__device__ __forceinline__ bf16x8 pp_frag(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

#define PP_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
// wait until at most `younger` K-steps of G LDS-DMA instructions each are still in flight
template <int G>
__device__ __forceinline__ void pp_wait(int younger) {
  static_assert(G == 3 || G == 4, "G");
  if constexpr (G == 4) {
    if (younger <= 0) PP_VM(0);
    else if (younger == 1) PP_VM(4);
    else if (younger == 2) PP_VM(8);
    else PP_VM(12);
  } else {
    if (younger <= 0) PP_VM(0);
    else if (younger == 1) PP_VM(3);
    else if (younger == 2) PP_VM(6);
    else if (younger == 3) PP_VM(9);
    else PP_VM(12);
  }
}
#undef PP_VM

// B-tile row r -> weight row.  SwiGLU: 16-row group g alternates gate (even g) and up (odd g) rows
// of output columns n_t * BN/2 + (g / 2) * 16 + r % 16.
template <int BN, bool SWIGLU>
__device__ __forceinline__ int pp_b_row(int r, int n_t, int half) {
  if (!SWIGLU) return n_t * BN + r;
  const int g = r >> 4;
  return ((g & 1) ? half : 0) + n_t * (BN / 2) + (g >> 1) * 16 + (r & 15);
}
}  // namespace

// MODE 0: C bf16 [M, N];  1: split-K slab P (f16 x 2^-6, common.h) [S, M, N];  2: SwiGLU C [M, N/2].
// VAR bit 0: weights nontemporal (read once); bit 1: grouped row-tile order (prefill, no split).
template <int BN, int MODE, int VAR>
__global__ void __launch_bounds__(512, 2) gemm_pp_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                         int K, int ks_per_split, int nsplit) {
  constexpr int BM = 256;
  constexpr int WM = BN == 256 ? 2 : 4, WN = 8 / WM;
  constexpr int TM = BM / WM, TN = BN / WN;            // wave tile: 128 x 64 or 64 x 64
  constexpr int RT = TM / 16, CT = TN / 16;            // 16 x 16 fragments per wave
  static_assert(CT == 4 && (RT == 4 || RT == 8), "wave tile");
  constexpr int PH = RT / 4;                           // phases per K-step (4 A x 4 B fragments each)
  constexpr int SLOT = (BM + BN) * PBK;                // bf16 elements per ring slot
  constexpr int NS = BN == 256 ? 5 : 6;
  constexpr int GA = BM * PBK / 512 / 8, GB = BN * PBK / 512 / 8;   // glds per wave per K-step
  constexpr int G = GA + GB, GP = G / PH;              // glds per wave per phase
  static_assert(G % PH == 0, "staging split");
  constexpr bool NT = (VAR & 1) != 0, GROUPED = (VAR & 2) != 0;
  constexpr bool SWIGLU = MODE == 2;
  constexpr int OUTW = SWIGLU ? BN / 2 : BN;           // output tile width (elements)
  constexpr int OPITCH = OUTW + 8;                     // LDS output row pitch (elements): +16 B
  static_assert(NS * SLOT * 2 <= 160 * 1024 && BM * OPITCH <= NS * SLOT, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wv >> 2;                             // ping-pong group: waves w and w+4 share a SIMD
  const int wm = BN == 256 ? (wv >> 2) : (wv >> 1), wn = BN == 256 ? (wv & 3) : (wv & 1);
  const int mtiles = (M + BM - 1) / BM;
  const int ntiles = SWIGLU ? (N / 2) / (BN / 2) : N / BN;
  const int total = gridDim.x;
  int b = blockIdx.x;
  {   // bijective XCD remap: consecutive logical blocks share an XCD
    const int q = total >> 3, r = total & 7, x = b & 7;
    b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (b >> 3);
  }
  int m_t, n_t, split;
  if constexpr (GROUPED) {
    const int per = 8 * ntiles, g = b / per, first = g * 8, gsz = min(mtiles - first, 8);
    m_t = first + (b % per) % gsz;
    n_t = (b % per) / gsz;
    split = 0;
  } else {
    m_t = b % mtiles;
    const int rest = b / mtiles;
    split = rest % nsplit;
    n_t = rest / nsplit;
  }
  const int m0 = m_t * BM;
  const int ks0 = split * ks_per_split;
  const int nt = max(0, min(K / PBK, ks0 + ks_per_split) - ks0);

  // staging sources: wave-instruction i covers 16 slot rows, lane -> (row 16 i + lane / 4,
  // physical chunk lane % 4) <- logical chunk pswz(row, lane % 4) of the source row
  const bf16* srcA[GA];
  const bf16* srcB[GB];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int r = 16 * (wv * GA + j) + (lane >> 2);
    srcA[j] = A + (size_t)min(m0 + r, M - 1) * K + (size_t)ks0 * PBK + pswz(r, lane & 3) * 8;
  }
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int r = 16 * (wv * GB + j) + (lane >> 2);
    srcB[j] = B + (size_t)pp_b_row<BN, SWIGLU>(r, n_t, N / 2) * K + (size_t)ks0 * PBK + pswz(r, lane & 3) * 8;
  }
  // piece p (0..G-1) of K-step ks into ring slot `slot`
  auto piece = [&](int slot, int ks, int p) {
    bf16* base = smem + slot * SLOT;
    if (p < GA)
      __builtin_amdgcn_global_load_lds((glb_vptr_p)(srcA[p] + ks * PBK), (lds_vptr_p)(base + (wv * GA + p) * 512), 16,
                                       0, 0);
    else
      __builtin_amdgcn_global_load_lds((glb_vptr_p)(srcB[p - GA] + ks * PBK),
                                       (lds_vptr_p)(base + BM * PBK + (wv * GB + p - GA) * 512), 16, 0, NT ? 2 : 0);
  };

  // fragment read offsets: lane (row l & 15, logical chunk l >> 4) of a 16-row fragment
  const uint32_t lane_off = (uint32_t)((lane & 15) * 64 + ((lane >> 4) ^ (((lane & 15) >> 1) & 3)) * 16);
  const uint32_t lds0 = (uint32_t)(size_t)(lds_vptr_p)smem + lane_off;
  const uint32_t a_off = (uint32_t)(wm * TM * 64), b_off = (uint32_t)(BM * 64 + wn * TN * 64);

  f32x4 acc[RT][CT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nt > 0) {
    // prologue: K-steps 0 .. NS-2 in flight, wait for K-step 0, one barrier for everyone
#pragma unroll
    for (int j = 0; j < NS - 1; ++j)
      if (j < nt) {
#pragma unroll
        for (int p = 0; p < G; ++p) piece(j, j, p);
      }
    pp_wait<G>(min(nt - 1, NS - 2));
    __builtin_amdgcn_s_barrier();
    if (grp == 1) __builtin_amdgcn_s_barrier();        // the stagger
    asm volatile("" ::: "memory");

    int slot = 0;                                      // ring slot of K-step t
    for (int t = 0; t < nt; ++t) {
      const uint32_t rb = lds0 + (uint32_t)(slot * SLOT * 2);
      const int islot = slot == 0 ? NS - 1 : slot - 1; // slot of K-step t + NS - 1 (= t - 1's)
      const int ks_issue = t + NS - 1;
      const bool more = t + 1 < nt;
      const int younger = min(nt - 2 - t, NS - 2);     // K-steps after t + 1 already issued
      bf16x8 fb[CT];
#pragma unroll
      for (int ph = 0; ph < PH; ++ph) {
        // ---- read section: this phase's staging pieces, fragments, (group 1) next K-step's wait
        if (ks_issue < nt) {
#pragma unroll
          for (int p = 0; p < GP; ++p) piece(islot, ks_issue, ph * GP + p);
        }
        bf16x8 fa[4];
        const uint32_t ra = rb + a_off + (uint32_t)(ph * 64 * 64);
        fa[0] = pp_frag<0>(ra);
        fa[1] = pp_frag<16 * 64>(ra);
        fa[2] = pp_frag<32 * 64>(ra);
        fa[3] = pp_frag<48 * 64>(ra);
        if (ph == 0) {
          const uint32_t rbb = rb + b_off;
          fb[0] = pp_frag<0>(rbb);
          fb[1] = pp_frag<16 * 64>(rbb);
          fb[2] = pp_frag<32 * 64>(rbb);
          fb[3] = pp_frag<48 * 64>(rbb);
        }
        if (ph == PH - 1 && more && grp == 1) pp_wait<G>(younger);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        // ---- MFMA section
#pragma unroll
        for (int ct = 0; ct < CT; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            acc[ph * 4 + r][ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[ct], fa[r], acc[ph * 4 + r][ct], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (ph == PH - 1 && more && grp == 0) pp_wait<G>(younger);
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
      }
      slot = slot == NS - 1 ? 0 : slot + 1;
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();        // balance the stagger
  }

  // ---- epilogue: accumulators -> LDS output image (8-byte writes) -> 16-byte row stores.
  // acc[rt][ct] lane l holds C[row wm*TM + rt*16 + (l & 15)][col wn*TN + ct*16 + 4*(l >> 4) + v]
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = wm * TM + rt * 16 + lr;
    if constexpr (SWIGLU) {
#pragma unroll
      for (int cp = 0; cp < CT / 2; ++cp) {
        const f32x4 g = acc[rt][2 * cp], u = acc[rt][2 * cp + 1];
        bf16x4 h;
#pragma unroll
        for (int v = 0; v < 4; ++v) h[v] = f2bf(silu_f(g[v]) * u[v]);
        const int col = wn * (TN / 2) + cp * 16 + 4 * lq;
        *reinterpret_cast<bf16x4*>(smem + row * OPITCH + col) = h;
      }
    } else {
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) {
        const int col = wn * TN + ct * 16 + 4 * lq;
        const f32x4 v = acc[rt][ct];
        if constexpr (MODE == 1) {
          f16x4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = (_Float16)(v[e] * kPartScale);
          *reinterpret_cast<f16x4*>(smem + row * OPITCH + col) = h;
        } else {
          bf16x4 h;
#pragma unroll
          for (int e = 0; e < 4; ++e) h[e] = f2bf(v[e]);
          *reinterpret_cast<bf16x4*>(smem + row * OPITCH + col) = h;
        }
      }
    }
  }
  __syncthreads();
  constexpr int CPR = OUTW / 8;                        // 16-byte chunks per output row
  constexpr int RPI = 512 / CPR;                       // rows per pass
  const int ch = tid % CPR, r0 = tid / CPR;
  const int ldc = SWIGLU ? N / 2 : N;
  const int col0 = n_t * OUTW + ch * 8;
#pragma unroll 4
  for (int r = r0; r < BM; r += RPI) {
    const int m = m0 + r;
    if (m >= M) break;
    const int4 v = *reinterpret_cast<const int4*>(smem + r * OPITCH + ch * 8);
    if constexpr (MODE == 1) {
      _Float16* Ph = reinterpret_cast<_Float16*>(P);
      *reinterpret_cast<int4*>(Ph + ((size_t)split * M + m) * N + col0) = v;
    } else {
      *reinterpret_cast<int4*>(C + (size_t)m * ldc + col0) = v;
    }
  }
}

// mode 0: C = A B^T;  mode 1: SwiGLU, C[M, N/2] = silu(A Bg^T) * (A Bu^T) with B = [Bg; Bu];
// mode 2: leave split-K partial slabs in ws (S > 1 required).  Returns the effective K slices S.
// variant bit 0: BN = 128 (else 256); bit 1: weights nontemporal; bit 2: grouped row-tile order
// (large M; ignored with a K split).
int gemm_pp(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
            int mode, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(K % PBK == 0 && K >= PBK, "K must be a positive multiple of 32");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  const int BN = (variant & 1) ? 128 : 256;
  const bool swiglu = mode == 1;
  DLLM_HOST_CHECK(N % BN == 0, "N must be a multiple of the column tile (128 / 256)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ksteps = K / PBK;
  const int kps = (ksteps + splits - 1) / splits;
  const int S = (ksteps + kps - 1) / kps;
  DLLM_HOST_CHECK(mode != 2 || S > 1, "mode 2 needs a K split");
  const int mtiles = (M + 255) / 256;
  const long grid = (long)(N / BN) * mtiles * S;
  DLLM_HOST_CHECK(grid >= 1 && grid < (1L << 31), "grid");
  const bool nt = (variant & 2) != 0;
  const bool grp = (variant & 4) != 0 && S == 1 && mtiles > 1;
#define DLLM_PP_GO(BN_, MODE_, VAR_)                                                                     \
  hipLaunchKernelGGL((gemm_pp_kernel<BN_, MODE_, VAR_>), dim3((unsigned)grid), dim3(512), 0, s, (const bf16*)a, \
                     (const bf16*)b, (bf16*)c, (float*)ws, M, N, K, kps, S)
#define DLLM_PP_V(BN_, MODE_)                                        \
  do {                                                               \
    if (grp) { if (nt) DLLM_PP_GO(BN_, MODE_, 3); else DLLM_PP_GO(BN_, MODE_, 2); } \
    else { if (nt) DLLM_PP_GO(BN_, MODE_, 1); else DLLM_PP_GO(BN_, MODE_, 0); }     \
  } while (0)
  if (S == 1) {
    if (BN == 256) { if (swiglu) DLLM_PP_V(256, 2); else DLLM_PP_V(256, 0); }
    else { if (swiglu) DLLM_PP_V(128, 2); else DLLM_PP_V(128, 0); }
    DLLM_HIP_CHECK(hipGetLastError());
    return 1;
  }
  DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  // split: natural column order slabs (a SwiGLU is applied by the reduce)
  if (BN == 256) DLLM_PP_V(256, 1);
  else DLLM_PP_V(128, 1);
#undef DLLM_PP_V
#undef DLLM_PP_GO
  DLLM_HIP_CHECK(hipGetLastError());
  if (mode == 2) return S;
  splitk_reduce_ex(c, ws, 0, S, M, N, swiglu ? 1 : 0, stream);
  return S;
}

}  // namespace dllm
