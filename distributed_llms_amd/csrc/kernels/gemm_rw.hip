// Register-weight decode GEMM for batch-sized M (<= 256): C[M,N] = A[M,K] . W[N,K]^T, bf16 in,
// f32 accumulate.  The engine's decode projections (qkv, o, gate|up + SwiGLU, down, LM head).
//
// Why (profiles/round3_gemm_experiments.md): at M = 256 a decode projection sits on the ridge
// between weight streaming and MFMA, and every LDS-staged design (gemm_wide, gemm_pp, and the
// retired gemm_gu) was capped at the same ~48 GB/s per CU -- the weight bytes in flight per CU were
// bounded by the LDS ring that also has to hold the (2x larger) activation tile.  Here the WEIGHTS
// never touch LDS:
//  * MFMA v_mfma_f32_32x32x16_bf16 with the weight as the A operand: lane l's A fragment is
//    W[row l & 31][k 16 j + 8 (l >> 5) ..+ 8] at k-step j -- one 16-byte buffer load straight into
//    4 VGPRs (default cache policy: nontemporal loads doubled the L2 requests, 106 vs 82 us on the
//    8B gate|up); from the nn.Linear layout that is 64 lanes in 64 rows, so the packed
//    fragment-major layout (PK below) is the fast form;
//  * each of the 4 waves (one per SIMD) owns 32 weight rows x all BM token rows (BM = 64 / 128 /
//    256 by M): BM / 32 accumulators of 32 x 32, every weight fragment feeds BM / 32 MFMAs;
//  * only the activations (L2-resident, shared by the 4 waves) are staged, by LDS-DMA
//    (buffer_load ... lds, 128-byte rows, 16-byte chunk swizzle c ^ ((row >> 1) & 7): conflict-free
//    fragment reads), in an NS-slot ring of BM x 64 K-tiles; the weight fragments of the K-tiles in
//    flight sit in NS register buffers (a smaller BM leaves LDS and registers for a deeper ring);
//  * ONE barrier per K-tile, before its last k-step: every wave has read the K-tile into registers
//    (its slot is re-staged from there), and the next K-tile has landed for every wave (counted
//    vmcnt -- weights and activations of a K-tile are issued together, 4 + BM / 32 VMEM ops per wave);
//  * per MFMA gap (24 free issue cycles behind a 32-cycle MFMA): 2 fragment reads of the next
//    k-step in the first half of a k-step's gaps, the VMEM ops (weight fragments, LDS-DMA pieces)
//    spread over the second halves, each MFMA waiting (counted lgkmcnt) only for the fragment it
//    consumes;
//  * epilogue straight from registers: a lane holds 4 consecutive output columns of one token row
//    per 4-register group -> 8-byte stores of bf16 / f16 split-K slabs; SwiGLU: the wave's 32
//    weight rows are 16 gate + 16 up rows of the same 16 outputs, so silu(g) * u is per lane;
//  * split-K over workgroups (slabs reduced by the next op, as gemm_wide), XCD-aware block order
//    (the workgroups of one XCD share a K slice of the activations in their L2).
#include "common.h"
#include "launchers.h"

#include <type_traits>
#include <utility>

namespace dllm {

namespace {
typedef __attribute__((address_space(3))) void* lds_vptr_r;
typedef int i32x4r __attribute__((ext_vector_type(4)));
constexpr int RBK = 64;                 // K per tile (4 k-steps of 16)

template <int... I, class F>
__device__ __forceinline__ void rw_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void rw_for(F&& f) {
  rw_for_impl(std::make_integer_sequence<int, N>{}, f);
}

template <int N>
__device__ __forceinline__ void rw_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}
// wait until at most `younger` K-tiles of RG ops each are still in flight (clamped to 0..MAXY),
// then tie the weight fragments w[0..3] the wait makes valid to an empty asm ("+v"): their loads
// are inline asm the compiler does not track, so nothing may read them before this point.  The
// counted waits take no operands and the tie is ONE statement after them: tied operands inside
// the branches made hipcc merge the values through copies placed BEFORE the wait (copies of
// registers still in flight).
template <int MAXY, int RG>
__device__ __forceinline__ void rw_wait_tiles(int younger, bf16x8 (&w)[4]) {
  static_assert(MAXY >= 0 && MAXY * RG <= 63, "vmcnt range");
  younger = younger < 0 ? 0 : (younger > MAXY ? MAXY : younger);
  rw_for<MAXY + 1>([&](auto y) {
    if (younger == y.value) rw_vm<y.value * RG>();
  });
  asm volatile("" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]));
}

// one weight fragment: 16 bytes per lane straight into VGPRs (buffer_load_dwordx4, voffset +
// soffset), in inline asm so that hipcc inserts no vmcnt waits of its own (its loop-carried
// scoreboard falls back to vmcnt(0)); validity comes from rw_wait_tiles
__device__ __forceinline__ void rw_wload(bf16x8& dst, uint32_t voff, const i32x4r& rs, int soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(dst) : "v"(voff), "s"(rs), "s"(soff));
}

template <int OFF>
__device__ __forceinline__ bf16x8 rw_frag(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}
// lgkmcnt(N) tied to the fragment the next MFMA consumes (N >= 16: no wait)
template <int N>
__device__ __forceinline__ void rw_lgkm(bf16x8& f) {
  if constexpr (N < 16) asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(f) : "i"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// the activation-fragment reads issued before MFMA mf of a k-step that are younger than fragment
// mf of the current set: the rest of the current set (read 2 per gap in the first MFR / 2 gaps of
// the previous k-step) + the next set's reads issued in this k-step so far
constexpr int rw_younger(int mfr, int mf) { return (mfr - 1 - mf) + 2 * (mf < mfr / 2 ? mf : mfr / 2); }
}  // namespace

// MODE 0: C bf16 [M, N];  1: split-K slab P [S, M, N] (natural column order, also for SwiGLU
// weights: the reducer applies silu(g) * u);  2: SwiGLU C [M, N / 2] from W = [Wg; Wu].
// BM: token rows per workgroup (>= M).  NS: activation ring slots = weight register buffers; the
// K-tiles t + 1 .. t + NS - 1 are in flight while K-tile t is multiplied.
// PK: W is stored FRAGMENT-MAJOR (ops/gemm.py pack_rw): 32-row group g, K-tile t, k-step j, lane L
// -> 16 bytes at ((g KT + t) 4 + j) 64 + L (16-byte units) = W[32 g + (L & 31)][64 t + 16 j +
// 8 (L >> 5) ..+ 8] (SwiGLU: group g = gate rows 16 g .. 16 g + 15, then the same up rows), so a
// wave's weight load is ONE contiguous KiB.  In the nn.Linear layout the 64 lanes of a load hit 64
// different 64-byte segments (rows 2 K bytes apart): 4x the L1 tag lookups of a coalesced load, and
// the L1 -- not HBM -- set the pace (profiles/round4_gemm_counters.md: TA stalled on it 25 M cycles
// vs 1 M for gemm_wide).
template <int BM, int NS, int MODE, bool SWROWS, bool PK>
__global__ void __launch_bounds__(256, 1) gemm_rw_kernel(const bf16* __restrict__ A, const bf16* __restrict__ W,
                                                         bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                         int K, int kts, int nsplit) {
  constexpr int MFR = BM / 32;            // 32-row token fragments per wave (= LDS-DMA pieces per wave)
  constexpr int AP = BM / 32;
  constexpr int RG = 4 + AP;              // VMEM ops per K-tile per wave
  constexpr int SLOT = BM * RBK * 2;      // bytes per activation slot
  static_assert(BM == 64 || BM == 128 || BM == 256, "BM");
  static_assert(NS >= 3 && NS * SLOT <= 160 * 1024 && (NS - 2) * RG <= 63, "ring");
  // VMEM schedule: the RG ops of one K-tile (4 weight fragments, then AP pieces) spread over the
  // NSL second-half gaps of a window's k-steps 0-2, in issue order
  constexpr int NSL = 3 * (MFR / 2);
  __shared__ __attribute__((aligned(16))) char smem[NS * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, r = lane & 31;
  const int ntiles = SWROWS ? (N / 2) / 64 : N / 128;
  int b = blockIdx.x;
  {   // bijective XCD remap: consecutive logical blocks share an XCD
    const int total = gridDim.x, q = total >> 3, rr = total & 7, x = b & 7;
    b = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + (b >> 3);
  }
  const int split = b / ntiles, n_t = b % ntiles;
  const int kt0 = split * kts;
  const int nt = min(K / RBK, kt0 + kts) - kt0;   // >= 1 (host: S = ceil(ktiles / kts))

  // weight row of lane row r (0..31) of this wave; SwiGLU rows: 16 gate rows then the 16 up rows of
  // the same outputs
  auto wrow_of = [&](int rr) {
    if constexpr (SWROWS) {
      const int f0 = n_t * 64 + wv * 16;
      return rr < 16 ? f0 + rr : N / 2 + f0 + rr - 16;
    } else {
      return n_t * 128 + wv * 32 + rr;
    }
  };
  const char* Wb = reinterpret_cast<const char*>(W) + (size_t)kt0 * RBK * 2;
  const char* Ab = reinterpret_cast<const char*>(A) + (size_t)kt0 * RBK * 2;
  i32x4r rsW;   // buffer descriptor of the weight slice: base, stride 0, byte range, raw dword format
  {
    const uint64_t wa = (uint64_t)(size_t)(PK ? reinterpret_cast<const char*>(W) : Wb);
    rsW[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)wa);
    rsW[1] = __builtin_amdgcn_readfirstlane((int)(uint32_t)(wa >> 32) & 0xffff);
    rsW[2] = __builtin_amdgcn_readfirstlane((int)((long)N * K * 2 - (PK ? 0L : (long)kt0 * RBK * 2)));
    rsW[3] = 0x00020000;
  }
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, (int)((long)M * K * 2 - (long)kt0 * RBK * 2), 0x00020000);
  const uint32_t woff = PK ? (uint32_t)(n_t * 4 + wv) * (uint32_t)(K / RBK * 4096) + (uint32_t)lane * 16
                           : (uint32_t)wrow_of(r) * (uint32_t)(K * 2) + (uint32_t)h * 16;

  // LDS-DMA pieces: piece q of wave wv fills slot rows 8 pi .. 8 pi + 7 (pi = AP wv + q), lane ->
  // (row 8 pi + lane / 8, physical chunk lane % 8) <- logical chunk (lane % 8) ^ swz(row)
  uint32_t offA[AP];
#pragma unroll
  for (int q = 0; q < AP; ++q) {
    const int row = 8 * (wv * AP + q) + (lane >> 3);
    const int srow = row < M ? row : M - 1;
    offA[q] = (uint32_t)srow * (uint32_t)(K * 2) + (uint32_t)(((lane & 7) ^ ((row >> 1) & 7)) * 16);
  }
  // fragment read offsets (bytes, within a slot) of k-step j: token row r of each 32-row m-frag
  // (the m-frag is the immediate offset 4096 mf), logical chunk 2 j + h
  const uint32_t lds0 = (uint32_t)(size_t)(lds_vptr_r)smem;
  uint32_t foff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) foff[j] = (uint32_t)(r * 128 + (((2 * j + h) ^ ((r >> 1) & 7)) * 16));

  f32x16 acc[MFR];
#pragma unroll
  for (int i = 0; i < MFR; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[i][e] = 0.f;
  bf16x8 wreg[NS][4];
  bf16x8 fs0[MFR], fs1[MFR];

  auto load_w = [&](bf16x8& dst, int t, int j) {
    if constexpr (PK) rw_wload(dst, woff + j * 1024, rsW, (kt0 + t) * 4096);
    else rw_wload(dst, woff + j * 32, rsW, t * (RBK * 2));
  };
  auto piece = [&](int slot, int t, int q) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_vptr_r)(smem + slot * SLOT + (wv * AP + q) * 1024), 16,
                                             (int)offA[q], t * (RBK * 2), 0, 0);
  };
  auto reads2 = [&](bf16x8 (&dst)[MFR], uint32_t addr, auto g) {   // fragments 2g, 2g + 1 of a k-step
    constexpr int G = decltype(g)::value;
    dst[2 * G] = rw_frag<(2 * G) * 4096>(addr);
    dst[2 * G + 1] = rw_frag<(2 * G + 1) * 4096>(addr);
  };
  // one k-step: MFR MFMAs on fragment set `cur` with weight fragment `wf`; gaps 0 .. MFR/2 - 1 read
  // the next k-step's fragments into `nxt` from LDS address `naddr` (if READ), the other gaps run
  // vm(gap - MFR / 2)
  auto kstep = [&](const bf16x8& wf, bf16x8 (&cur)[MFR], bf16x8 (&nxt)[MFR], uint32_t naddr, auto rd, auto waits,
                   auto&& vm) {
    constexpr bool READ = decltype(rd)::value, WAIT = decltype(waits)::value;
    rw_for<MFR>([&](auto mf) {
      constexpr int MF = decltype(mf)::value;
      if constexpr (WAIT) rw_lgkm<rw_younger(MFR, MF)>(cur[MF]);
      acc[MF] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf, cur[MF], acc[MF], 0, 0, 0);
      if constexpr (MF < MFR / 2) {
        if constexpr (READ) reads2(nxt, naddr, mf);
      } else {
        vm(std::integral_constant<int, MF - MFR / 2>{});
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  auto no_vm = [](auto) {};

  // ---- prologue: K-tiles 0 .. NS-2 (each: its 4 weight fragments, then its AP LDS-DMA pieces).
  // Straight-line: a K-tile past the slice (nt < NS - 1, short K slices only) is a dummy copy of
  // K-tile nt - 1 into a buffer / slot nothing reads -- it only makes the waits below more
  // conservative
  rw_for<NS - 1>([&](auto p) {
    const int tp = min((int)p.value, nt - 1);
#pragma unroll
    for (int j = 0; j < 4; ++j) load_w(wreg[p.value][j], tp, j);
#pragma unroll
    for (int q = 0; q < AP; ++q) piece(p.value, tp, q);
  });
  rw_wait_tiles<NS - 2, RG>(NS - 2, wreg[0]);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  rw_for<MFR / 2>([&](auto g) { reads2(fs0, lds0 + foff[0], g); });   // K-tile 0, k-step 0
  __builtin_amdgcn_sched_barrier(0);

  // ---- window t (I = t mod NS): the 4 k-steps of K-tile t (weight buffer I, slot t mod NS);
  // K-tile u = t + NS - 1 is issued during k-steps 0-2 (weights into buffer u mod NS = buffer of
  // K-tile t - 1, pieces into slot u mod NS = slot of K-tile t - 1, both free since window t - 1);
  // barrier B_t before k-step 3: K-tile t + 1 has landed for every wave (counted vmcnt: the K-tiles
  // issued after it, min(NS - 2, nt - 2 - t), stay in flight) and every wave holds K-tile t's
  // fragments; k-step 3 reads K-tile t + 1's first fragments.  Only the VMEM issue is
  // predicated: the MFMA and fragment-read stream is the same in every window (the last window's
  // trailing reads fetch stale LDS bytes nobody uses), so no register merges in the loop.
  auto window = [&](int t, auto ic) {
    constexpr int I = decltype(ic)::value, IU = (I + NS - 1) % NS;
    const int s0 = t % NS, s1 = (t + 1) % NS, su = (t + NS - 1) % NS;
    const uint32_t b0 = lds0 + (uint32_t)(s0 * SLOT), b1 = lds0 + (uint32_t)(s1 * SLOT);
    const int tu = t + NS - 1;
    const bool issue = tu < nt;
    // the VMEM ops whose schedule slot is (k-step j, second-half gap x)
    auto ops = [&](auto jc, auto x) {
      constexpr int SL = decltype(jc)::value * (MFR / 2) + decltype(x)::value;
      rw_for<RG>([&](auto oc) {
        constexpr int O = decltype(oc)::value;
        if constexpr (O * NSL / RG == SL) {
          if (issue) {
            if constexpr (O < 4) load_w(wreg[IU][O], tu, O);
            else piece(su, tu, O - 4);
          }
        }
      });
    };
    kstep(wreg[I][0], fs0, fs1, b0 + foff[1], std::true_type{}, std::true_type{},
          [&](auto x) { ops(std::integral_constant<int, 0>{}, x); });
    kstep(wreg[I][1], fs1, fs0, b0 + foff[2], std::true_type{}, std::true_type{},
          [&](auto x) { ops(std::integral_constant<int, 1>{}, x); });
    kstep(wreg[I][2], fs0, fs1, b0 + foff[3], std::true_type{}, std::true_type{},
          [&](auto x) { ops(std::integral_constant<int, 2>{}, x); });
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    rw_wait_tiles<NS - 2, RG>(nt - 2 - t, wreg[(I + 1) % NS]);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    kstep(wreg[I][3], fs1, fs0, b1 + foff[0], std::true_type{}, std::false_type{}, no_vm);
  };

  // groups of NS windows: every weight buffer index is a compile-time constant
  for (int t0 = 0; t0 < nt; t0 += NS) {
    rw_for<NS>([&](auto i) {
      if (t0 + i.value < nt) window(t0 + i.value, i);
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // ---- epilogue: acc[mf] register 4 g + i = row 8 g + 4 h + i of the wave's 32 weight rows,
  // token mf * 32 + r
#pragma unroll
  for (int mf = 0; mf < MFR; ++mf) {
    const int m = mf * 32 + r;
    if (m >= M) continue;
    if constexpr (MODE == 2) {
      const int f = n_t * 64 + wv * 16 + 4 * h;
      bf16x4 o0, o1;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o0[i] = f2bf(silu_f(acc[mf][i]) * acc[mf][8 + i]);
        o1[i] = f2bf(silu_f(acc[mf][4 + i]) * acc[mf][12 + i]);
      }
      bf16* row = C + (size_t)m * (N / 2);
      *reinterpret_cast<bf16x4*>(row + f) = o0;
      *reinterpret_cast<bf16x4*>(row + f + 8) = o1;
    } else {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = wrow_of(8 * g + 4 * h);
        if constexpr (MODE == 0) {
          bf16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = f2bf(acc[mf][4 * g + i]);
          *reinterpret_cast<bf16x4*>(C + (size_t)m * N + n) = o;
        } else {
          const size_t idx = ((size_t)split * M + m) * N + n;
#if DLLM_PART_TYPE == 2
          f16x4 o;
#pragma unroll
          for (int i = 0; i < 4; ++i) o[i] = (_Float16)(acc[mf][4 * g + i] * kPartScale);
          *reinterpret_cast<f16x4*>(reinterpret_cast<_Float16*>(P) + idx) = o;
#else
#pragma unroll
          for (int i = 0; i < 4; ++i) part_store(P, idx + i, acc[mf][4 * g + i]);
#endif
        }
      }
    }
  }
}

static int rw_bm(int M) { return M <= 64 ? 64 : M <= 128 ? 128 : 256; }
static int rw_default_ns(int bm) { return bm == 256 ? 4 : bm == 128 ? 6 : 8; }

// mode 0: C = A W^T;  mode 1: SwiGLU, C[M, N/2] = silu(A Wg^T) * (A Wu^T) with W = [Wg; Wu];
// mode 2: leave split-K partial slabs in ws (no reduce; S > 1 required).
// variant: bits 0-3 ring slots NS (0 = the row tile's default: 4 / 6 / 8 at 256 / 128 / 64 rows;
// 256 rows: 3..5, 128: 4 / 6 / 8, 64: 4 / 8), bit 4: W is fragment-major packed (see PK), bits
// 8-9: row tile override (1 = 64, 2 = 128, 3 = 256).
// Returns the effective number of K slices S.
int gemm_rw(uintptr_t c, uintptr_t a, uintptr_t w, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
            int mode, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1 && M <= 256, "gemm_rw serves 1 <= M <= 256");
  DLLM_HOST_CHECK(K % RBK == 0 && K >= RBK, "K must be a positive multiple of 64");
  DLLM_HOST_CHECK(mode == 0 || mode == 1 || mode == 2, "mode");
  DLLM_HOST_CHECK(N % 128 == 0, "N must be a multiple of 128");
  DLLM_HOST_CHECK((long)N * K * 2 < (1L << 31) && (long)M * K * 2 < (1L << 31), "operands must be < 2 GiB");
  DLLM_HOST_CHECK(splits >= 1, "splits >= 1");
  const int bmo = (variant >> 8) & 3;
  const int bm = bmo == 1 ? 64 : bmo == 2 ? 128 : bmo == 3 ? 256 : rw_bm(M);
  DLLM_HOST_CHECK(M <= bm, "row tile override smaller than M");
  const int ns = (variant & 15) ? (variant & 15) : rw_default_ns(bm);
  DLLM_HOST_CHECK(bm != 256 || (ns >= 3 && ns <= 5), "ring slots at 256 rows: 3..5");
  DLLM_HOST_CHECK(bm != 128 || ns == 4 || ns == 6 || ns == 8, "ring slots at 128 rows: 4, 6, 8");
  DLLM_HOST_CHECK(bm != 64 || ns == 4 || ns == 8, "ring slots at 64 rows: 4, 8");
  const bool pk = (variant & 16) != 0;
  const bool swiglu = mode == 1;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int ktiles = K / RBK;
  const int kts = (ktiles + splits - 1) / splits;
  const int S = (ktiles + kts - 1) / kts;
  DLLM_HOST_CHECK(mode != 2 || S > 1, "mode 2 needs a K split");
  if (S > 1) DLLM_HOST_CHECK(ws != 0 && (long)S * M * N <= ws_floats, "split-K workspace too small");
  const int ntiles = swiglu ? (N / 2) / 64 : N / 128;
  const long grid = (long)ntiles * S;
  const int kmode = S == 1 ? (swiglu ? 2 : 0) : 1;
#define DLLM_RW_GO(BM_, NS_, MODE_, SW_, PK_)                                                               \
  hipLaunchKernelGGL((gemm_rw_kernel<BM_, NS_, MODE_, SW_, PK_>), dim3((unsigned)grid), dim3(256), 0, s,    \
                     (const bf16*)a, (const bf16*)w, (bf16*)c, (float*)ws, M, N, K, kts, S)
#define DLLM_RW_MODES1(BM_, NS_, PK_)                                         \
  do {                                                                        \
    if (kmode == 2) DLLM_RW_GO(BM_, NS_, 2, true, PK_);                       \
    else if (kmode == 0) DLLM_RW_GO(BM_, NS_, 0, false, PK_);                 \
    else if (swiglu) DLLM_RW_GO(BM_, NS_, 1, true, PK_);                      \
    else DLLM_RW_GO(BM_, NS_, 1, false, PK_);                                 \
  } while (0)
#define DLLM_RW_MODES(BM_, NS_)                                               \
  do {                                                                        \
    if (pk) DLLM_RW_MODES1(BM_, NS_, true);                                   \
    else DLLM_RW_MODES1(BM_, NS_, false);                                     \
  } while (0)
  if (bm == 256) {
    if (ns == 3) DLLM_RW_MODES(256, 3);
    else if (ns == 5) DLLM_RW_MODES(256, 5);
    else DLLM_RW_MODES(256, 4);
  } else if (bm == 128) {
    if (ns == 4) DLLM_RW_MODES(128, 4);
    else if (ns == 8) DLLM_RW_MODES(128, 8);
    else DLLM_RW_MODES(128, 6);
  } else {
    if (ns == 4) DLLM_RW_MODES(64, 4);
    else DLLM_RW_MODES(64, 8);
  }
#undef DLLM_RW_MODES
#undef DLLM_RW_MODES1
#undef DLLM_RW_GO
  DLLM_HIP_CHECK(hipGetLastError());
  if (S == 1 || mode == 2) return S;
  splitk_reduce_ex(c, ws, 0, S, M, N, swiglu ? 1 : 0, stream);
  return S;
}

}  // namespace dllm
