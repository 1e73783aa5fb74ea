// 4-wave software-pipelined MFMA GEMM for 256-row tiles: C[M,N] = A[M,K] . B[N,K]^T, bf16 in, f32
// accumulate.  The engine runs the prefill MLP gate|up through it (schedule 2, 256-column tiles,
// grouped row-tile order, SwiGLU fused into the epilogue: faster than hipBLASLt + silu_mul,
// profiles/round3_gemm_experiments.md); decode-M split-K forms are kept for experiments.
//
// Why this shape (profiles/round3_gemm_counters.md): hipBLASLt's 256 x 256 kernel keeps the MFMA
// pipe ~82 % busy with ONE wave per SIMD and a 128 x 128 wave tile, while 8-wave designs that
// synchronise twice per 16-MFMA phase (the 2-waves-per-SIMD ping-pong this file first held, the
// lock-step gemm_wide) reach ~62 %: a workgroup barrier every 256 MFMA cycles costs more than the
// partner wave hides.  Here:
//  * tile 256 x BN, 4 waves as 2 x 2, wave tile 128 x BN/2 (8 x 8 or 8 x 4 accumulators of
//    v_mfma_f32_16x16x32_bf16: up to 256 accumulator registers, one wave per SIMD);
//  * 64-deep K-tiles in an LDS ring (BN 256: 2 x 64 KiB, BN 128: 3 x 48 KiB), filled by
//    global_load_lds_dwordx4 in full 128-byte rows (8 rows per wave-instruction), the 16-byte
//    chunk swizzle c ^ ((row >> 1) & 7) on the per-lane SOURCE address and on the fragment read
//    (conflict-free ds_read_b128; rule 21);
//  * ONE barrier per K-tile, in its middle: K-half 0's MFMAs run while K-half 1's fragments are
//    read; at the barrier every read of the tile is done and the next tile has landed (counted
//    vmcnt, never 0 in the loop at BN 128); K-half 1's MFMAs run while the next tile's K-half 0 is
//    read and the tile NB ahead is staged into the slot just freed -- fragment reads and LDS-DMA
//    pieces interleave with the MFMAs in program order (sched_barrier), so the wave's own MFMA
//    stream covers their latency;
//  * operands swapped in the MFMA (B fragment first), so a lane's accumulator holds 4 CONSECUTIVE
//    output columns of one row: the epilogue packs them 8 bytes at a time into an LDS image of the
//    output tile (padded rows, conflict-free), then every lane stores 16-byte row chunks --
//    full 128-byte lines for bf16 outputs, f16 split-K slabs and the SwiGLU product alike;
//  * SwiGLU without a weight permutation: the B tile's 16-row groups alternate gate / up rows of
//    the fused [2I, K] weight, so gate and up of an output column meet in one lane.
#include "common.h"
#include "launchers.h"

#include <atomic>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <utility>

namespace dllm {

namespace {
constexpr int PBK = 64;                       // K per ring slot (128-byte rows)
typedef __attribute__((address_space(3))) void* lds_vptr_p;
typedef __attribute__((address_space(1))) void* glb_vptr_p;

__device__ __forceinline__ int pswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int OFF>
__device__ __forceinline__ bf16x8 pp_frag(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(addr), "i"(OFF));
  return r;
}

// fragment read at an LDS byte address, in inline asm: hipcc does not count it, so the only waits
// are the counted ones of PpSched (its own waitcnt insertion falls back to lgkmcnt(0) at the loop
// head and before every MFMA that uses a read from the previous iteration)
__device__ __forceinline__ bf16x8 pp_frag_dyn(uint32_t addr) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(addr));
  return r;
}

#define PP_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
// wait until at most `younger` K-steps of G LDS-DMA instructions each are still in flight
template <int G>
__device__ __forceinline__ void pp_wait_n(int younger) {   // younger: compile-time after inlining
  static_assert(G == 12 || G == 16, "G");
  if (younger <= 0) PP_VM(0);
  else if constexpr (G == 12) { if (younger == 1) PP_VM(12); else PP_VM(24); }
  else { if (younger == 1) PP_VM(16); else PP_VM(32); }
}
#undef PP_VM

// s_waitcnt vmcnt(N) for a compile-time N
template <int N>
__device__ __forceinline__ void pp_vm() {
  static_assert(N >= 0 && N <= 63, "vmcnt");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// f(integral_constant<int, i>) for i = 0 .. N-1, each i a constant expression
template <int... I, class F>
__device__ __forceinline__ void pp_static_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void pp_static_for(F&& f) {
  pp_static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// s_waitcnt lgkmcnt(N) for a compile-time N (16 = no wait); a sched_barrier keeps hipcc from
// hoisting register-only MFMAs above an inline-asm wait (guide rule 18)
template <int N>
__device__ __forceinline__ void pp_lgkm() {
  static_assert(N >= 0 && N <= 16, "lgkmcnt");
  if constexpr (N < 16) {
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(N) : "memory");
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Fragment-read schedule of one K-half (RT A-fragments, CT B-fragments; MFMA i uses A r = i / CT,
// B c = i % CT).  The reads for the OTHER K-half go out after MFMA pos(): A fragment a right after
// its register's last MFMA in this K-half (a * CT + CT - 1), B fragment b spread over the first
// half of the stream; in K-half 1 nothing before the barrier at EB - 1.  wait_before(h, i): the
// lgkmcnt that makes MFMA i of K-half h wait for exactly its operands' reads (issued during the
// previous K-half), counting the younger reads of that K-half and this K-half's reads so far.
template <int RT, int CT>
struct PpSched {
  static constexpr int NMF = RT * CT, EB = CT, BE = (NMF / 2) / CT > 0 ? (NMF / 2) / CT : 1;
  static constexpr int pos(int half, int kind, int k) {
    if (kind == 0) return k * CT + CT - 1 > (half ? EB - 1 : -1) ? k * CT + CT - 1 : EB - 1;
    return half == 0 ? k * BE : EB - 1 + k * BE;
  }
  static constexpr int key(int half, int kind, int k) { return pos(half, kind, k) * 64 + kind * 32 + k; }
  static constexpr int younger(int half, int kind, int k) {   // reads of `half` issued after (kind, k)
    int n = 0;
    for (int a = 0; a < RT; ++a) n += key(half, 0, a) > key(half, kind, k);
    for (int b = 0; b < CT; ++b) n += key(half, 1, b) > key(half, kind, k);
    return n;
  }
  static constexpr int issued_before(int half, int i) {        // this K-half's reads before MFMA i
    int n = 0;
    for (int a = 0; a < RT; ++a) n += pos(half, 0, a) < i;
    for (int b = 0; b < CT; ++b) n += pos(half, 1, b) < i;
    return n;
  }
  static constexpr int wait_before(int half, int i) {
    const int r = i / CT, c = i % CT, prev = 1 - half;
    // the first MFMA of a row needs its A fragment, the first row needs every B fragment
    const bool need_a = c == 0, need_b = r == 0;
    if (!need_a && !need_b) return 16;
    int n = 1 << 20;
    if (need_a) n = younger(prev, 0, r);
    if (need_b) { const int nb = younger(prev, 1, c); n = nb < n ? nb : n; }
    n += issued_before(half, i);
    return n > 15 ? 15 : n;
  }
};

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
__global__ void __launch_bounds__(256, 1) gemm_pp_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         bf16* __restrict__ C, float* __restrict__ P, int M, int N,
                                                         int K, int ks_per_split, int nsplit, float* __restrict__ D,
                                                         const int* __restrict__ gather, const int* __restrict__ counts,
                                                         const int* __restrict__ offsets, int E) {
  constexpr int NW = 4, NWN = 2;
  constexpr int BM = 256, TM = 128, TN = BN / NWN;     // waves as 2 (M) x NWN (N)
  constexpr int RT = TM / 16, CT = TN / 16;            // 16 x 16 fragments per wave: 8 x 8 or 8 x 4
  constexpr int SLOT = (BM + BN) * PBK;                // bf16 elements per ring slot (one K-tile)
  constexpr int NB = BN == 256 ? 2 : 3;                // K-tiles held in LDS
  constexpr int GA = BM * PBK * 2 / 1024 / NW, GB = BN * PBK * 2 / 1024 / NW;  // glds per wave per K-tile
  constexpr int G = GA + GB;
  constexpr bool NT = (VAR & 1) != 0, GROUPED = (VAR & 2) != 0;
  constexpr bool PROF = (VAR & 4) != 0;                // diagnostic build: cycle stamps around B_t
  // diagnostic ablations (wrong results, timing only): no LDS-DMA pieces / no fragment reads in the loop
  constexpr bool NOLOAD = (VAR & 8) != 0, NOREAD = (VAR & 16) != 0;
  // schedule 2 (VAR 32): a K-tile's fragments are all read into registers early in its first K-half,
  // so its slot is re-staged from then on -- LDS-DMA pieces spread over ~60 % of the K-tile instead
  // of bunched into half of K-half 1 (see the loop)
  constexpr bool SCHED2 = (VAR & 32) != 0;
  constexpr bool SWIGLU = MODE == 2;
  constexpr int OUTW = SWIGLU ? BN / 2 : BN;           // output tile width (elements)
  // schedule 2 + SwiGLU: the epilogue stages gate and up as bf16 (the image is the full BN wide)
  // and applies silu(g) * u while storing -- the fused fp32 form kept the accumulators live
  // longer and made hipcc shuffle them through VGPRs inside the main loop
  constexpr bool SWI2 = SWIGLU && SCHED2;
  constexpr int IMGW = SWI2 ? BN : OUTW;               // LDS image width (elements)
  constexpr int OPITCH = IMGW + 8;                     // LDS output row pitch (elements): +16 B
  constexpr int SMEM = NB * SLOT > BM * OPITCH ? NB * SLOT : BM * OPITCH;   // ring, then output image
  static_assert(SMEM * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 smem[SMEM];

  [[maybe_unused]] unsigned long long rt_entry = 0, rt_loop0 = 0, rt_loop1 = 0;
  if constexpr (PROF) rt_entry = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / NWN, wn = wv % NWN;
  // MOE (VAR 128): grouped expert GEMM -- the row tiles of every expert's segment of the
  // expert-sorted slot space, counts / offsets read on the device (no host sync); the grid holds an
  // upper bound of row tiles (slots / 256 + E), the surplus workgroups exit at once
  constexpr bool MOE = (VAR & 128) != 0;
  const int ntiles = N / BN;
  const int mtiles = MOE ? (int)(gridDim.x / ntiles) : (M + BM - 1) / BM;
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
  // the tile's rows: [r0, min(r0 + BM, rcnt)) of the row range that starts at slot roff (dense:
  // roff 0, rows m0 .. M); MOE: expert ex's segment, its weight We = B + ex N K
  int r0 = m0, rcnt = M, roff = 0;
  const bf16* We = B;
  if constexpr (MOE) {
    int base = 0, ex = -1;
    for (int x = 0; x < E; ++x) {
      const int c = counts[x], nx = (c + BM - 1) / BM;
      if (ex < 0 && m_t < base + nx) {
        ex = x;
        r0 = (m_t - base) * BM;
        rcnt = c;
      }
      base += nx;
    }
    if (ex < 0) return;                                // past the last real row tile (uniform)
    roff = offsets[ex];
    We = B + (size_t)ex * N * K;
  }
  const int ks0 = split * ks_per_split;
  const int nt = max(0, min(K / PBK, ks0 + ks_per_split) - ks0);

  // staging sources: wave-instruction i covers 8 slot rows, lane -> (row 8 i + lane / 8,
  // physical chunk lane % 8) <- logical chunk pswz(row, lane % 8) of the source row.  Byte
  // offsets are 32-bit from a wave-uniform base (operands < 4 GiB, checked on the host): one VGPR
  // per A piece (rows past M clamp to M - 1) and ONE for every B piece -- a B piece's row is a
  // uniform function of the piece index plus lane / 8, also for the SwiGLU row interleave
  const char* Ab = reinterpret_cast<const char*>(A) + (size_t)ks0 * PBK * 2;
  const char* Bb = reinterpret_cast<const char*>(We) + (size_t)ks0 * PBK * 2;
  // the swizzle of row 8 q + lane / 8 depends on q's parity: ((8 q + x) >> 1) & 7 = (4 q + x / 2) & 7
  uint32_t chunk_q[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) chunk_q[par] = (uint32_t)(pswz(8 * par + (lane >> 3), lane & 7) * 16);
  uint32_t offA[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int q = wv * GA + j, r = 8 * q + (lane >> 3);
    int srow;
    if constexpr (MOE) {
      const int slot = roff + min(r0 + r, rcnt - 1);
      srow = gather ? gather[slot] : slot;
    } else {
      srow = min(m0 + r, M - 1);
    }
    offA[j] = (uint32_t)srow * (uint32_t)(K * 2) + chunk_q[q & 1];
  }
  uint32_t offB[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) offB[par] = (uint32_t)(lane >> 3) * (uint32_t)(K * 2) + chunk_q[par];
  // piece p (0..G-1) of K-tile ks into ring slot `slot`.  ks >= nt (past this split's range):
  // a DUMMY piece -- K-tile nt - 1 again (L2-resident), into a slot nobody reads again -- so that
  // every K-tile of the loop issues exactly G pieces: straight-line MFMA streams and static vmcnt
  // counts
  // schedule 2 stages through buffer loads: a 32-bit per-lane offset + an SGPR offset per piece
  // (K-tile, B row group), so no 64-bit VGPR address math in the MFMA stream (register pressure)
  [[maybe_unused]] __amdgpu_buffer_rsrc_t rsA, rsB;
  if constexpr (SCHED2) {
    rsA = __builtin_amdgcn_make_buffer_rsrc((void*)Ab, (short)0, (int)((long)M * K * 2 - (long)ks0 * 128), 0x00020000);
    rsB = __builtin_amdgcn_make_buffer_rsrc((void*)Bb, (short)0, (int)((long)N * K * 2 - (long)ks0 * 128), 0x00020000);
  }
  auto piece = [&](int slot, int ks, int p) {
    bf16* base = smem + slot * SLOT;
    ks = min(ks, nt - 1);                              // wave-uniform: SALU, no per-lane select
    if constexpr (SCHED2) {
      if (p < GA) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_vptr_p)(base + (wv * GA + p) * 512), 16, (int)offA[p],
                                                 ks * PBK * 2, 0, 0);
      } else {
        const int q = wv * GB + p - GA;
        const int brow = pp_b_row<BN, SWIGLU>(8 * q, n_t, N / 2);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_vptr_p)(base + BM * PBK + q * 512), 16, (int)offB[q & 1],
                                                 brow * K * 2 + ks * PBK * 2, 0, NT ? 2 : 0);
      }
      return;
    }
    if (p < GA) {
      __builtin_amdgcn_global_load_lds((glb_vptr_p)(Ab + offA[p] + ks * PBK * 2),
                                       (lds_vptr_p)(base + (wv * GA + p) * 512), 16, 0, 0);
    } else {
      const int q = wv * GB + p - GA;                  // 8-row group of the B tile
      const int brow = pp_b_row<BN, SWIGLU>(8 * q, n_t, N / 2);   // row of lane 0 (uniform)
      __builtin_amdgcn_global_load_lds((glb_vptr_p)(Bb + (size_t)brow * K * 2 + offB[q & 1] + ks * PBK * 2),
                                       (lds_vptr_p)(base + BM * PBK + q * 512), 16, 0, NT ? 2 : 0);
    }
  };

  // fragment read offsets: lane (row l & 15, logical chunk 4 kh + (l >> 4)) of a 16-row fragment
  // in K-half kh; the swizzle of rows r0 + x (r0 % 16 == 0) depends on x only
  const uint32_t lds_base = (uint32_t)(size_t)(lds_vptr_p)smem;
  uint32_t lane_off[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
    lane_off[kh] = (uint32_t)((lane & 15) * 128 + ((4 * kh + (lane >> 4)) ^ (((lane & 15) >> 1) & 7)) * 16);
  const uint32_t a_off = (uint32_t)(wm * TM * 128), b_off = (uint32_t)(BM * 128 + wn * TN * 128);

  f32x4 acc[RT][CT];
#pragma unroll
  for (int i = 0; i < RT; ++i)
#pragma unroll
    for (int j = 0; j < CT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of one K-half: fa[RT] (A rows of the wave tile), fb[CT] (B rows); two sets, so
  // the next K-half's reads are in flight under this one's MFMAs (software pipeline)
  bf16x8 fa0[RT], fb0[CT], fa1[RT], fb1[CT];

  if constexpr (SCHED2) {
  if (nt > 0) {
    // ---- schedule 2.  Per K-tile t (slot cur = t % NB), MFMA i = 0 .. 2 NMF - 1 (K-half h = i / NMF):
    //  * set 0 (fa0, fb0) = K-half 0 fragments, read at the end of the previous K-tile; the first
    //    MFMA of each row waits with a COUNTED lgkmcnt for exactly its A fragment (row 0: all B);
    //  * the K-half 1 fragments (set 1) are read from cur one every 2 MFMAs from the start; after
    //    MFMA IB1 (< NMF): lgkmcnt(0) + barrier -> every wave holds the whole K-tile in registers,
    //    slot cur is free, and the G pieces of K-tile t + NB are staged into it one every GE MFMAs;
    //  * after MFMA IB3 (>= NMF, set 0 no longer in use): vmcnt(pieces younger than K-tile t + 1's)
    //    + barrier -> K-tile t + 1 has landed for every wave; its K-half 0 fragments are read into
    //    set 0 one every 2 MFMAs.
    constexpr int NMF = RT * CT, NR = RT + CT;
    constexpr int IB1 = 2 * NR + 8 < NMF - 1 ? 2 * NR + 8 : NMF - 1;
    constexpr int GE = (2 * NMF - 4 - IB1 - 1) / G > 1 ? (2 * NMF - 4 - IB1 - 1) / G : 1;
    constexpr int IB3 = 2 * NMF - 8 - 2 * NR > NMF ? 2 * NMF - 8 - 2 * NR : NMF;
    constexpr int PB3 = (IB3 - IB1 - 1) / GE + 1 < G ? (IB3 - IB1 - 1) / GE + 1 : G;   // pieces issued by IB3
    constexpr int VC = (NB - 2) * G + PB3;
    static_assert(IB1 + 1 + GE * (G - 1) < 2 * NMF && IB3 + 1 + 2 * (NR - 1) < 2 * NMF, "schedule 2 fits a K-tile");
    static_assert(VC <= 63, "vmcnt");
    // fragment reads off two base registers per set (A rows, B rows of the slot) with the
    // fragment's offset in the instruction's immediate field: no address math per read
    auto rd0 = [&](uint32_t base, auto mc) {           // set-0 read m: B fragments first, then A rows
      constexpr int m = decltype(mc)::value;
      if constexpr (m < CT) fb0[m] = pp_frag<m * 16 * 128>(base + b_off);
      else fa0[m - CT] = pp_frag<(m - CT) * 16 * 128>(base + a_off);
    };
    auto rd1 = [&](uint32_t base, auto mc) {
      constexpr int m = decltype(mc)::value;
      if constexpr (m < CT) fb1[m] = pp_frag<m * 16 * 128>(base + b_off);
      else fa1[m - CT] = pp_frag<(m - CT) * 16 * 128>(base + a_off);
    };
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int p = 0; p < G; ++p) piece(j, j, p);
    pp_vm<(NB - 1) * G>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    [[maybe_unused]] unsigned long long st0 = 0, rt0 = 0, sb0 = 0, sb1 = 0, sb3 = 0;
    if constexpr (PROF) {   // stamped before the counted reads (an s_memtime counts on lgkmcnt)
      rt0 = __builtin_amdgcn_s_memrealtime();
      rt_loop0 = rt0;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st0) :: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    pp_static_for<NR>([&](auto mc) { rd0(lds_base + lane_off[0], mc); });
    __builtin_amdgcn_sched_barrier(0);
    int slot = 0;
    for (int t = 0; t < nt; ++t) {
      const int nslot = slot == NB - 1 ? 0 : slot + 1;
      const uint32_t base1 = lds_base + (uint32_t)(slot * SLOT * 2) + lane_off[1];
      const uint32_t base0 = lds_base + (uint32_t)(nslot * SLOT * 2) + lane_off[0];
      pp_static_for<2 * NMF>([&](auto ic) {
        constexpr int i = decltype(ic)::value, h = i / NMF, j = i % NMF, r = j / CT, c = j % CT;
        if constexpr (h == 0 && c == 0) {
          constexpr int w0 = (RT - 1 - r) + (j / 2 < NR ? j / 2 : NR);
          pp_lgkm<(w0 > 15 ? 15 : w0)>();
        }
        if constexpr (h == 0)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[c], fa0[r], acc[r][c], 0, 0, 0);
        else
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[c], fa1[r], acc[r][c], 0, 0, 0);
        if constexpr (i % 2 == 1 && i / 2 < NR) {
          if constexpr (!NOREAD) rd1(base1, std::integral_constant<int, i / 2>{});
        }
        if constexpr (i == IB1) {
          if constexpr (PROF) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sb0) :: "memory");
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
          if constexpr (PROF) {
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long s1;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(s1) :: "memory");
            sb1 += s1 - sb0;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if constexpr (i > IB1 && (i - IB1 - 1) % GE == 0 && (i - IB1 - 1) / GE < G) {
          if constexpr (!NOLOAD) piece(slot, t + NB, (i - IB1 - 1) / GE);
        }
        if constexpr (i == IB3) {
          if constexpr (PROF) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sb0) :: "memory");
          pp_vm<VC>();
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
          if constexpr (PROF) {
            __builtin_amdgcn_sched_barrier(0);
            unsigned long long s1;
            asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(s1) :: "memory");
            sb3 += s1 - sb0;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        if constexpr (i > IB3 && (i - IB3 - 1) % 2 == 0 && (i - IB3 - 1) / 2 < NR) {
          if constexpr (!NOREAD) rd0(base0, std::integral_constant<int, (i - IB3 - 1) / 2>{});
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      slot = nslot;
    }
    if constexpr (PROF) {
      unsigned long long st1;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st1) :: "memory");
      const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      rt_loop1 = rt1;
      const float vals[6] = {(float)(st1 - st0), (float)(sb1 + sb3), (float)nt, (float)(rt1 - rt0), (float)sb1,
                             (float)sb3};
      float* rec = D + ((size_t)blockIdx.x * 4 + wv) * 128;
      if (lane < 6) rec[lane < 4 ? lane : lane + 16] = vals[lane < 6 ? lane : 0];
    }
  }
  } else {
  if (nt > 0) {
    using SC = PpSched<RT, CT>;
    constexpr int NMF = RT * CT;                       // 64 or 32 MFMAs per K-half
    // prologue: K-tiles 0 .. NB-1 in flight; wait for K-tile 0; read K-half 0 of it in the
    // order a K-half 1 issues its reads (so the counted waits of the first K-half 0 hold)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int p = 0; p < G; ++p) piece(j, j, p);
    pp_wait_n<G>(NB - 1);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    {
      const uint32_t base = lds_base + lane_off[0];
#pragma unroll
      for (int i = 0; i < NMF; ++i) {
#pragma unroll
        for (int r = 0; r < RT; ++r)
          if (SC::pos(1, 0, r) == i) fa0[r] = pp_frag_dyn(base + a_off + r * 16 * 128);
#pragma unroll
        for (int c = 0; c < CT; ++c)
          if (SC::pos(1, 1, c) == i) fb0[c] = pp_frag_dyn(base + b_off + c * 16 * 128);
      }
      __builtin_amdgcn_sched_barrier(0);
    }

    // One K-half: NMF MFMAs, row-fragment-major, with the other K-half's fragment reads and (in
    // K-half 1) the LDS-DMA pieces interleaved in program order.  Every MFMA that first uses a
    // fragment waits with a COUNTED lgkmcnt for exactly that read (PpSched), never lgkmcnt(0)
    // inside the stream.  K-half 1 holds the K-tile's one barrier after its first fragment row:
    // the last reads of this slot have had a row of MFMAs to land (WAR), the next tile has
    // landed for every wave (RAW), and only then are the next tile's fragments read and this
    // slot re-staged.
    int slot = 0;                                      // ring slot of K-tile t
    [[maybe_unused]] unsigned long long st0 = 0, sbt = 0, sbt0 = 0, rt0 = 0;
    if constexpr (PROF) {
      rt0 = __builtin_amdgcn_s_memrealtime();
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st0) :: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    for (int t = 0; t < nt; ++t) {
      const uint32_t cur = lds_base + (uint32_t)(slot * SLOT * 2);
      const int nslot = slot == NB - 1 ? 0 : slot + 1;
      const uint32_t nxt = lds_base + (uint32_t)(nslot * SLOT * 2);
      // ---- K-half 0: MFMAs on (fa0, fb0); read K-half 1 of this K-tile into (fa1, fb1)
      {
        const uint32_t base = cur + lane_off[1];
        pp_static_for<NMF>([&](auto ic) {
          constexpr int i = decltype(ic)::value, r = i / CT, c = i % CT;
          pp_lgkm<SC::wait_before(0, i)>();
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[c], fa0[r], acc[r][c], 0, 0, 0);
#pragma unroll
          for (int a = 0; a < RT; ++a)
            if (!NOREAD && SC::pos(0, 0, a) == i) fa1[a] = pp_frag_dyn(base + a_off + a * 16 * 128);
#pragma unroll
          for (int b = 0; b < CT; ++b)
            if (!NOREAD && SC::pos(0, 1, b) == i) fb1[b] = pp_frag_dyn(base + b_off + b * 16 * 128);
          __builtin_amdgcn_sched_barrier(0);
        });
      }
      // ---- K-half 1: MFMAs on (fa1, fb1); after its first row the barrier B_t, then read K-half 0
      // of K-tile t + 1 into (fa0, fb0) (garbage past the last tile, never used) and stage K-tile
      // t + NB into this slot (a dummy piece past the range): straight-line, no branch
      {
        const uint32_t base = nxt + lane_off[0];
        constexpr int GE = 2;                          // one LDS-DMA piece every 2 MFMAs after B_t
        pp_static_for<NMF>([&](auto ic) {
          constexpr int i = decltype(ic)::value, r = i / CT, c = i % CT;
          pp_lgkm<SC::wait_before(1, i)>();
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[c], fa1[r], acc[r][c], 0, 0, 0);
          if constexpr (i == SC::EB - 1) {
            // B_t: every read of this slot done (WAR), K-tile t + 1 landed for every wave (RAW)
            if constexpr (PROF)
              asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(sbt0) :: "memory");
            else
              asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            pp_wait_n<G>(NB - 2);
            __builtin_amdgcn_sched_barrier(0);
            __builtin_amdgcn_s_barrier();
            if constexpr (PROF) {
              __builtin_amdgcn_sched_barrier(0);
              unsigned long long s1;
              asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(s1) :: "memory");
              sbt += s1 - sbt0;
              __builtin_amdgcn_sched_barrier(0);
            }
          }
          if constexpr (i >= SC::EB - 1 && (i - SC::EB + 1) % GE == 0 && (i - SC::EB + 1) / GE < G)
            if constexpr (!NOLOAD) piece(slot, t + NB, (i - SC::EB + 1) / GE);
#pragma unroll
          for (int a = 0; a < RT; ++a)
            if (!NOREAD && SC::pos(1, 0, a) == i) fa0[a] = pp_frag_dyn(base + a_off + a * 16 * 128);
#pragma unroll
          for (int b = 0; b < CT; ++b)
            if (!NOREAD && SC::pos(1, 1, b) == i) fb0[b] = pp_frag_dyn(base + b_off + b * 16 * 128);
          __builtin_amdgcn_sched_barrier(0);
        });
      }
      slot = nslot;
    }
    if constexpr (PROF) {   // per wave: loop cycles, cycles in B_t (counter waits + barrier), K-tiles, 100 MHz ticks
      unsigned long long st1;
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st1) :: "memory");
      const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_s_waitcnt(0xC07F);
      const float vals[4] = {(float)(st1 - st0), (float)sbt, (float)nt, (float)(rt1 - rt0)};
      float* rec = D + ((size_t)blockIdx.x * 4 + wv) * 128;
      if (lane < 4) rec[lane] = vals[lane & 3];
    }
  }
  }
  // ---- epilogue: accumulators -> LDS output image (8-byte writes) -> 16-byte row stores.
  // acc[rt][ct] lane l holds C[row wm*TM + rt*16 + (l & 15)][col wn*TN + ct*16 + 4*(l >> 4) + v]
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int lr = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    const int row = wm * TM + rt * 16 + lr;
    if constexpr (SWIGLU && !SWI2) {
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
  constexpr int RPI = 64 * NW / CPR;                   // rows per pass
  const int ch = tid % CPR, rs0 = tid / CPR;
  const int ldc = SWIGLU ? N / 2 : N;
  const int col0 = n_t * OUTW + ch * 8;
  // SWI2: output columns 8 ch .. 8 ch + 7 sit in 16-column group ch / 2 -> gate at image column
  // 32 (ch / 2) + 8 (ch % 2), up 16 further
  const int icol = SWI2 ? 32 * (ch >> 1) + 8 * (ch & 1) : ch * 8;
#pragma unroll 4
  for (int r = rs0; r < BM; r += RPI) {
    if (r0 + r >= rcnt) break;
    const int m = roff + r0 + r;
    int4 v = *reinterpret_cast<const int4*>(smem + r * OPITCH + icol);
    if constexpr (SWI2) {
      const bf16x8 g = *reinterpret_cast<const bf16x8*>(&v);
      const bf16x8 u = *reinterpret_cast<const bf16x8*>(smem + r * OPITCH + icol + 16);
      bf16x8 h;
#pragma unroll
      for (int e = 0; e < 8; ++e) h[e] = f2bf(silu_f(bf2f(g[e])) * bf2f(u[e]));
      v = *reinterpret_cast<const int4*>(&h);
    }
    if constexpr (MODE == 1) {
      _Float16* Ph = reinterpret_cast<_Float16*>(P);
      *reinterpret_cast<int4*>(Ph + ((size_t)split * M + m) * N + col0) = v;
    } else {
      *reinterpret_cast<int4*>(C + (size_t)m * ldc + col0) = v;
    }
  }
  if constexpr (PROF && SCHED2) {   // timeline of this wave (100 MHz ticks) + where it ran
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long rt_end = __builtin_amdgcn_s_memrealtime();
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)\n\ts_getreg_b32 %1, hwreg(HW_REG_XCC_ID)" : "=s"(hw), "=s"(xcc));
    const double v8[6] = {(double)rt_entry, (double)rt_loop0, (double)rt_loop1, (double)rt_end, (double)hw, (double)xcc};
    double* rec = reinterpret_cast<double*>(D + ((size_t)blockIdx.x * 4 + wv) * 128 + 8);
    if (lane < 6) rec[lane] = v8[lane < 6 ? lane : 0];
  }
}

// mode 0: C = A B^T;  mode 1: SwiGLU, C[M, N/2] = silu(A Bg^T) * (A Bu^T) with B = [Bg; Bu];
// mode 2: leave split-K partial slabs in ws (S > 1 required).  Returns the effective K slices S.
// variant bit 0: BN = 128 (else 256); bit 1: weights nontemporal; bit 2: grouped row-tile order
// (large M; ignored with a K split).
int gemm_pp(uintptr_t c, uintptr_t a, uintptr_t b, uintptr_t ws, long ws_floats, int M, int N, int K, int splits,
            int mode, int variant, uintptr_t stream) {
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(K % PBK == 0 && K >= PBK, "K must be a positive multiple of 64");
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
  DLLM_HOST_CHECK((long)M * K * 2 < (1L << 32) && (long)N * K * 2 < (1L << 32), "operands must be < 4 GiB");
  DLLM_HOST_CHECK(grid >= 1 && grid < (1L << 31), "grid");
  const bool nt = (variant & 2) != 0;
  const bool grp = (variant & 4) != 0 && S == 1 && mtiles > 1;
#define DLLM_PP_GO(BN_, MODE_, VAR_)                                                                     \
  hipLaunchKernelGGL((gemm_pp_kernel<BN_, MODE_, VAR_>), dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)a, \
                     (const bf16*)b, (bf16*)c, (float*)ws, M, N, K, kps, S, dbg, (const int*)nullptr,       \
                     (const int*)nullptr, (const int*)nullptr, 0)
  // variant bit 6: schedule 2 (the K-tile's fragments read early, staging spread; weights
  // nontemporal with bit 1 only in the natural tile order).  Bit 3: diagnostic build -- per-wave cycle stamps (loop, B_t waits) into the LAST
  // grid x 512 floats of ws (after the slabs); output as usual.  With it (schedule 1 only), bit 4:
  // no LDS-DMA pieces in the loop, bit 5: no fragment reads in the loop (ablations: wrong results,
  // timing only)
  const bool sched2 = (variant & 64) != 0;
  const bool prof = (variant & 8) != 0;
  float* dbg = nullptr;
  if (prof) {
    DLLM_HOST_CHECK(ws != 0 && grid * 512 + (S > 1 ? (long)S * M * N : 0) <= ws_floats, "profile build: ws too small");
    dbg = (float*)ws + (ws_floats - grid * 512);
  }
#define DLLM_PP_V(BN_, MODE_)                                        \
  do {                                                               \
    if (sched2) {                                                    \
      if (prof) { if (grp) DLLM_PP_GO(BN_, MODE_, 38); else DLLM_PP_GO(BN_, MODE_, 36); } \
      else if (grp) DLLM_PP_GO(BN_, MODE_, 34);                      \
      else if (nt) DLLM_PP_GO(BN_, MODE_, 33);                       \
      else DLLM_PP_GO(BN_, MODE_, 32);                               \
    } else if (prof) {                                               \
      if (grp) DLLM_PP_GO(BN_, MODE_, 6);                            \
      else if (variant & 16) DLLM_PP_GO(BN_, MODE_, 12);             \
      else if (variant & 32) DLLM_PP_GO(BN_, MODE_, 20);             \
      else DLLM_PP_GO(BN_, MODE_, 4);                                \
    }                                                                \
    else if (grp) { if (nt) DLLM_PP_GO(BN_, MODE_, 3); else DLLM_PP_GO(BN_, MODE_, 2); } \
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

// Grouped expert GEMM over the expert-sorted slot space (MoE prefill): expert e owns
// slots [offsets[e], offsets[e] + counts[e]) (device arrays, never read on the host); its rows are
// x[gather[slot]] (gather null: x[slot]) and its weight W[e] ([N, K]; SwiGLU: [2I, K] = [Wg; Wu]).
// y [slots, N] (SwiGLU: [slots, N / 2]).  Schedule 2, 256 x 256 tiles, grouped row-tile order.
// xrows: rows of x (buffer range), slots: total slot count (grid bound: slots / 256 + E row tiles).
void gemm_pp_moe(uintptr_t y, uintptr_t x, uintptr_t gather, uintptr_t w, uintptr_t counts, uintptr_t offsets, int E,
                 int N, int K, int xrows, int slots, int mode, uintptr_t stream) {
  DLLM_HOST_CHECK(E >= 1 && E <= 256, "1 <= experts <= 256");
  DLLM_HOST_CHECK(K % PBK == 0 && K >= PBK, "K must be a positive multiple of 64");
  DLLM_HOST_CHECK(N % 256 == 0, "N must be a multiple of 256");
  DLLM_HOST_CHECK(mode == 0 || mode == 1, "mode 0 (plain) or 1 (SwiGLU)");
  DLLM_HOST_CHECK(xrows >= 1 && slots >= 1, "rows");
  DLLM_HOST_CHECK((long)xrows * K * 2 < (1L << 32) && (long)N * K * 2 < (1L << 32), "operands must be < 4 GiB");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const long grid = (long)(N / 256) * ((slots + 255) / 256 + E);
  DLLM_HOST_CHECK(grid < (1L << 31), "grid");
  if (mode == 1)
    hipLaunchKernelGGL((gemm_pp_kernel<256, 2, 128 | 32 | 2>), dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)x,
                       (const bf16*)w, (bf16*)y, (float*)nullptr, xrows, N, K, K / PBK, 1, (float*)nullptr,
                       (const int*)gather, (const int*)counts, (const int*)offsets, E);
  else
    hipLaunchKernelGGL((gemm_pp_kernel<256, 0, 128 | 32 | 2>), dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)x,
                       (const bf16*)w, (bf16*)y, (float*)nullptr, xrows, N, K, K / PBK, 1, (float*)nullptr,
                       (const int*)gather, (const int*)counts, (const int*)offsets, E);
  DLLM_HIP_CHECK(hipGetLastError());
}

// ---- Persistent prefill GEMM (gemm_pf): schedule 2's K-tile body, one workgroup per CU walking
// its share of the 256 x 256 output tiles, the LDS-DMA pipeline CONTINUOUS across tile boundaries.
//
// Why (profiles/round3_gemm_experiments.md, per-CU timeline of schedule 2 at M = 8192): the loop
// ran 92.5 % of the time -- every 256 x 256 tile paid a 4.3 us epilogue through an LDS image (the
// ring cannot be restaged while the image occupies it), a prologue that waits for two K-tiles from
// HBM, and a workgroup relaunch.  Here the pieces of the NEXT tile's first K-tiles are staged by the
// current tile's last K-tiles exactly as any other K-tile (a tile boundary is invisible to the
// ring), and the epilogue stores straight from the accumulators (a lane holds 4 consecutive output
// columns of one row: 8-byte stores, 32 contiguous bytes per row and fragment, merged into full
// lines in L2 by the same wave's neighbouring fragments), so no LDS, no barrier and no wait for the
// ring is on the tile boundary -- only the stores' issue and the accumulator reset.
//
// Tile order: the grouped order of gemm_pp (8 row tiles x all column tiles per group), walked as
// tile = w + i P by P = gridDim.x workgroups, w the XCD-aware rank (workgroup b runs on XCD b % 8;
// w = (b % 8) (P / 8) + b / 8), so each XCD's L2 serves 32 consecutive tiles of the grouped order
// (8 row tiles x 4 column tiles) at a time.
// MODE 0: C bf16 [M, N];  2: SwiGLU C [M, N / 2] with B = [Bg; Bu] (row groups as pp_b_row).
// SCH 8: nontemporal output stores (large SwiGLU outputs), else 0.  The schedule sweeps of rounds 3-5
// (barrier positions, piece spacing, row-group widths, and the split A / B LDS release of round 5,
// all within 0.5 % of this schedule: profiles/round5_raw/r5d_pf_sched.txt) were removed.
struct PfSched {
  int ib1, ib3, ge, gm;
};

// ---- gemm_pf's dynamic tile queue (DYN).  The grouped tile order is cut into chunks of PF_CH
// consecutive tiles (8 row tiles x 4 column tiles); chunk c belongs to XCD c % 8, whose workgroups
// pull its tiles in order from the XCD's head counter (one 128-byte line each) and, when it is
// empty, steal from the other XCDs' heads.  A workgroup that starts late -- its CU held by a
// co-resident kernel, e.g. an RCCL receive spinning on its LDS -- finds the tiles taken and exits,
// instead of owning a static share (tile = w + i P) that the whole GEMM then waits for.  The last
// workgroup to retire resets the heads for the next launch on the stream.
// queue layout (ints): head of XCD x at [32 x], retire counter at [256].
constexpr int PF_CH = 32;
constexpr int PF_QUEUE_INTS = 9 * 32;

__device__ __forceinline__ int pf_count(int x, int tiles) {         // tiles of XCD x's partition
  const int nch = (tiles + PF_CH - 1) / PF_CH;
  if (x >= nch) return 0;
  const int cx = (nch - 1 - x) / 8 + 1, last = x + 8 * (cx - 1);
  return (cx - 1) * PF_CH + min(PF_CH, tiles - last * PF_CH);
}

__device__ __forceinline__ int pf_tau(int x, int j) { return (x + 8 * (j / PF_CH)) * PF_CH + j % PF_CH; }

// blocking fetch (lane 0): the XCD's own head first, then the others'; -1 = no tile left
__device__ int pf_fetch(int* q, int xcd, int tiles, int first_try = -1) {
#pragma unroll 1
  for (int k = 0; k < 8; ++k) {
    const int x = (xcd + k) & 7, n = pf_count(x, tiles);
    if (n == 0) continue;
    int j;
    if (k == 0 && first_try >= 0) {
      j = first_try;                                                // the asynchronous fetch's result
    } else {
      if (__hip_atomic_load(q + 32 * x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= n) continue;
      j = atomicAdd(q + 32 * x, 1);
    }
    if (j < n) return pf_tau(x, j);
  }
  return -1;
}

// the K loop's fetch: issued in inline asm, so hipcc inserts no wait for it; the counted vmcnt
// wait of the NEXT K-tile (every LDS-DMA piece of that K-tile is younger) covers its return
__device__ __forceinline__ int pf_fetch_async(int* head) {
  int old;
  asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(old) : "v"(head), "v"(1) : "memory");
  return old;
}

__device__ void pf_retire(int* q, int grid) {                      // lane 0, once per workgroup
  if (atomicAdd(q + 256, 1) == grid - 1) {
#pragma unroll
    for (int x = 0; x < 8; ++x) __hip_atomic_store(q + 32 * x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(q + 256, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}
// {barrier after set-1 reads (MFMA), barrier before set-0 reads, MFMAs between pieces (0 = spread
// over the rest of the K-tile), row tiles per group of the tile order}
constexpr PfSched kPfSched{40, 88, 0, 8};

template <int MODE, int SCH = 0, bool DYN = false>
__global__ void __launch_bounds__(256, 1) gemm_pf_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                         bf16* __restrict__ C, int M, int N, int K,
                                                         int* __restrict__ queue) {
  constexpr int NW = 4, NWN = 2, BM = 256, BN = 256, TM = 128, TN = BN / NWN;
  constexpr int RT = TM / 16, CT = TN / 16;            // 8 x 8 accumulators per wave
  constexpr int SLOT = (BM + BN) * PBK, NB = 2;        // 2 x 64 KiB ring
  constexpr int GA = BM * PBK * 2 / 1024 / NW, GB = BN * PBK * 2 / 1024 / NW, G = GA + GB;
  constexpr bool SWIGLU = MODE == 2;
  constexpr int OUTW = SWIGLU ? BN / 2 : BN;           // output tile width (elements)
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  __shared__ __attribute__((aligned(16))) bf16 smem[NB * SLOT];
  __shared__ int tq[4];                                // DYN: tile of local ordinal i at [i & 3]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wv / NWN, wn = wv % NWN;
  const int ldc = SWIGLU ? N / 2 : N;
  const int mtiles = (M + BM - 1) / BM;
  const int ntn = N / BN, tiles = ntn * mtiles;
  const int P = gridDim.x;                             // a multiple of 8 (host)
  const int w = (int)(blockIdx.x & 7) * (P >> 3) + (int)(blockIdx.x >> 3);
  const int xcd = (int)(blockIdx.x & 7);               // blocks are dealt round-robin over the XCDs
  int mine = 0;                                        // static: my tile count
  if constexpr (DYN) {
    if (tid == 0) {
      const int t0 = pf_fetch(queue, xcd, tiles);
      tq[0] = t0;
      tq[1] = t0 >= 0 ? pf_fetch(queue, xcd, tiles) : -1;
    }
    __syncthreads();
    if (tq[0] < 0) {                                   // uniform: every tile already taken
      if (tid == 0) pf_retire(queue, P);
      return;
    }
  } else {
    mine = w < tiles ? (tiles - 1 - w) / P + 1 : 0;
    if (mine == 0) return;                             // uniform: before any load or barrier
  }
  constexpr int GM = kPfSched.gm;                      // row tiles per group of the tile order
  const int nt = K / PBK, per = GM * ntn;
  auto tile_of = [&](int i) { return DYN ? tq[i & 3] : w + i * P; };   // my i-th tile (grouped order)
  auto tile_mn = [&](int tau, int& m_t, int& n_t) {
    const int g = tau / per, first = g * GM, gsz = min(mtiles - first, GM), q = tau - g * per;
    m_t = first + q % gsz;
    n_t = q / gsz;
  };

  // ---- staging side: tile s_i's K-tile s_kt; per-lane A row offsets of that tile (rows past M
  // clamp to M - 1), B rows through the SGPR offset (uniform per piece)
  const __amdgpu_buffer_rsrc_t rsA =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, (int)(unsigned)((long)M * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsB =
      __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, (int)(unsigned)((long)N * K * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsC =
      __builtin_amdgcn_make_buffer_rsrc((void*)C, (short)0, (int)(unsigned)((long)M * ldc * 2), 0x00020000);
  uint32_t chunk_q[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) chunk_q[par] = (uint32_t)(pswz(8 * par + (lane >> 3), lane & 7) * 16);
  uint32_t offB[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) offB[par] = (uint32_t)(lane >> 3) * (uint32_t)(K * 2) + chunk_q[par];
  uint32_t offA[GA];
  int s_i = 0, s_kt = 0, s_n = 0;
  int pend = -1, pend_i = 0;                           // DYN (lane 0): fetch in flight, its ordinal
  auto set_stage = [&](int tau) {
    int m_t, n_t;
    tile_mn(tau, m_t, n_t);
    s_n = n_t;
    const int r0 = m_t * BM;
#pragma unroll
    for (int j = 0; j < GA; ++j) {
      const int q = wv * GA + j, r = 8 * q + (lane >> 3);
      offA[j] = (uint32_t)min(r0 + r, M - 1) * (uint32_t)(K * 2) + chunk_q[q & 1];
    }
  };
  // piece p of the staging K-tile into ring slot `slot`
  auto piece = [&](int slot, int p) {
    bf16* base = smem + slot * SLOT;
    if (p < GA) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (lds_vptr_p)(base + (wv * GA + p) * 512), 16, (int)offA[p],
                                               s_kt * PBK * 2, 0, 0);
    } else {
      const int q = wv * GB + p - GA;
      const uint32_t brow = (uint32_t)pp_b_row<BN, SWIGLU>(8 * q, s_n, N / 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (lds_vptr_p)(base + BM * PBK + q * 512), 16, (int)offB[q & 1],
                                               (int)(brow * (uint32_t)(K * 2) + (uint32_t)(s_kt * PBK * 2)),
                                               0, 0);
    }
  };
  // next staging K-tile; past my last tile: K-tile nt - 1 of it again (a DUMMY piece into a slot
  // nobody reads again, so every K-tile issues exactly G pieces: static vmcnt counts)
  // DYN: the staging side moving onto ordinal s_i issues the fetch of ordinal s_i + 1 (lane 0,
  // asynchronous); the next advance(), one K-tile and one counted vmcnt wait later, resolves it
  // into tq -- read by every wave at the following tile switch, at least one K-tile (two barriers)
  // later (nt >= 2, host check)
  auto advance = [&]() {
    if constexpr (DYN) {
      if (tid == 0 && pend_i > 0) {
        asm volatile("" : "+v"(pend));              // not before this point (the vmcnt wait above)
        tq[pend_i & 3] = pf_fetch(queue, xcd, tiles, pend);
        pend_i = 0;
      }
    }
    if (++s_kt == nt) {
      const bool more = DYN ? tq[(s_i + 1) & 3] >= 0 : s_i + 1 < mine;
      if (more) {
        ++s_i;
        s_kt = 0;
        set_stage(tile_of(s_i));
        if constexpr (DYN) {
          if (tid == 0) {
            if (pf_count(xcd, tiles) > 0) {
              pend = pf_fetch_async(queue + 32 * xcd);
            } else {
              pend = 1 << 30;                          // no own partition: resolve by stealing
            }
            pend_i = s_i + 1;
          }
        }
      } else {
        s_kt = nt - 1;
      }
    }
  };

  const uint32_t lds_base = (uint32_t)(size_t)(lds_vptr_p)smem;
  uint32_t lane_off[2];
#pragma unroll
  for (int kh = 0; kh < 2; ++kh)
    lane_off[kh] = (uint32_t)((lane & 15) * 128 + ((4 * kh + (lane >> 4)) ^ (((lane & 15) >> 1) & 7)) * 16);
  const uint32_t a_off = (uint32_t)(wm * TM * 128), b_off = (uint32_t)(BM * 128 + wn * TN * 128);

  f32x4 acc[RT][CT];
  bf16x8 fa0[RT], fb0[CT], fa1[RT], fb1[CT];
  constexpr int NMF = RT * CT, NR = RT + CT;
  constexpr PfSched SC = kPfSched;
  constexpr int IB1 = SC.ib1;
  constexpr int GE = SC.ge ? SC.ge : ((2 * NMF - 4 - IB1 - 1) / G > 1 ? (2 * NMF - 4 - IB1 - 1) / G : 1);
  constexpr int IB3 = SC.ib3;
  static_assert(IB1 > 2 * NR - 1 && IB1 < NMF && IB3 >= NMF, "schedule 2 barriers");
  constexpr int PB3 = (IB3 - IB1 - 1) / GE + 1 < G ? (IB3 - IB1 - 1) / GE + 1 : G;
  constexpr int VC = (NB - 2) * G + PB3;
  static_assert(IB1 + 1 + GE * (G - 1) < 2 * NMF && IB3 + 1 + 2 * (NR - 1) < 2 * NMF, "schedule 2 fits a K-tile");
  static_assert(VC <= 63, "vmcnt");
  auto rd0 = [&](uint32_t base, auto mc) {
    constexpr int m = decltype(mc)::value;
    if constexpr (m < CT) fb0[m] = pp_frag<m * 16 * 128>(base + b_off);
    else fa0[m - CT] = pp_frag<(m - CT) * 16 * 128>(base + a_off);
  };
  auto rd1 = [&](uint32_t base, auto mc) {
    constexpr int m = decltype(mc)::value;
    if constexpr (m < CT) fb1[m] = pp_frag<m * 16 * 128>(base + b_off);
    else fa1[m - CT] = pp_frag<(m - CT) * 16 * 128>(base + a_off);
  };

  // prologue: the first NB K-tiles of my first tile in flight, K-tile 0 landed, its K-half 0 read
  set_stage(tile_of(0));
#pragma unroll
  for (int j = 0; j < NB; ++j) {
#pragma unroll
    for (int p = 0; p < G; ++p) piece(j, p);
    advance();
  }
  pp_vm<(NB - 1) * G>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  pp_static_for<NR>([&](auto mc) { rd0(lds_base + lane_off[0], mc); });
  __builtin_amdgcn_sched_barrier(0);

  const int lr = lane & 15, lq = lane >> 4;
  int slot = 0;
  for (int ti = 0; DYN ? ti <= s_i : ti < mine; ++ti) {   // DYN: s_i > ti once staging moved on
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
      for (int j = 0; j < CT; ++j) {
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+a"(acc[i][j]));            // zeroed in place, in AGPRs
      }
    for (int t = 0; t < nt; ++t) {
      // schedule 2's K-tile (gemm_pp_kernel): set-1 reads from the start, barrier after MFMA IB1
      // (slot free), pieces of the staging K-tile one every GE MFMAs, counted vmcnt + barrier after
      // MFMA IB3 (next K-tile landed -- across a tile boundary too), next K-half 0 reads
      const int nslot = slot == NB - 1 ? 0 : slot + 1;
      const uint32_t base1 = lds_base + (uint32_t)(slot * SLOT * 2) + lane_off[1];
      const uint32_t base0 = lds_base + (uint32_t)(nslot * SLOT * 2) + lane_off[0];
      pp_static_for<2 * NMF>([&](auto ic) {
        constexpr int i = decltype(ic)::value, h = i / NMF, j = i % NMF, r = j / CT, c = j % CT;
        if constexpr (h == 0 && c == 0) {
          constexpr int w0 = (RT - 1 - r) + (j / 2 < NR ? j / 2 : NR);
          pp_lgkm<(w0 > 15 ? 15 : w0)>();
        }
        if constexpr (h == 0)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[c], fa0[r], acc[r][c], 0, 0, 0);
        else
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb1[c], fa1[r], acc[r][c], 0, 0, 0);
        if constexpr (i % 2 == 1 && i / 2 < NR) rd1(base1, std::integral_constant<int, i / 2>{});
        if constexpr (i == IB1) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (i > IB1 && (i - IB1 - 1) % GE == 0 && (i - IB1 - 1) / GE < G) piece(slot, (i - IB1 - 1) / GE);
        if constexpr (i == IB3) {
          pp_vm<VC>();
          __builtin_amdgcn_sched_barrier(0);
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (i > IB3 && (i - IB3 - 1) % 2 == 0 && (i - IB3 - 1) / 2 < NR)
          rd0(base0, std::integral_constant<int, (i - IB3 - 1) / 2>{});
        __builtin_amdgcn_sched_barrier(0);
      });
      advance();
      slot = nslot;
    }
    // epilogue straight from the accumulators: acc[r][c] lane l = C[row wm TM + 16 r + (l & 15)]
    // [col wn TN + 16 c + 4 (l >> 4) + v] (SwiGLU: fragments 2 cp (gate) and 2 cp + 1 (up) hold the
    // same output columns).  Two fragments' bf16 quads per lane are exchanged between 16-lane rows
    // (v_permlane16_swap: row 1 <-> row 0's partner, row 3 <-> row 2's) so that every lane holds 8
    // consecutive columns: 16-byte stores, a row's 16 lanes covering 64 contiguous bytes.  Buffer
    // stores, rows past M dropped by the range check (offset 0x80000000): no branch to hoist
    // accumulator reads over.
    int m_t, n_t;
    tile_mn(tile_of(ti), m_t, n_t);
    const uint32_t colb = (uint32_t)(n_t * OUTW + wn * (OUTW / NWN) + 16 * (lq & 1) + 8 * (lq >> 1)) * 2;
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      // pin row r's accumulators in AGPRs up to here: hipcc would otherwise copy all 256 to VGPRs
      // at the K loop's exit (and spill, draining the pipeline with vmcnt(0) waits)
#pragma unroll
      for (int c = 0; c < CT; ++c) asm volatile("" : "+a"(acc[r][c]));
      const int row = m_t * BM + wm * TM + r * 16 + lr;
      const uint32_t vo = row < M ? (uint32_t)row * (uint32_t)(ldc * 2) + colb : 0x80000000u;
      constexpr int NQ = SWIGLU ? CT / 2 : CT;         // bf16 quads per lane in this row group
      u32x2 q[NQ];
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        bf16x4 hq;
        if constexpr (SWIGLU) {
          const f32x4 g = acc[r][2 * i], u = acc[r][2 * i + 1];
#pragma unroll
          for (int v = 0; v < 4; ++v) hq[v] = f2bf(silu_f(g[v]) * u[v]);
        } else {
#pragma unroll
          for (int v = 0; v < 4; ++v) hq[v] = f2bf(acc[r][i][v]);
        }
        q[i] = __builtin_bit_cast(u32x2, hq);
      }
#pragma unroll
      for (int pr = 0; pr < NQ / 2; ++pr) {
        u32x2 x = q[2 * pr], y = q[2 * pr + 1];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto sw = __builtin_amdgcn_permlane16_swap(x[d], y[d], false, false);
          x[d] = sw[0];
          y[d] = sw[1];
        }
        const u32x4 o = {x[0], x[1], y[0], y[1]};
        // SCH 8 (SwiGLU outputs larger than the Infinity Cache): nontemporal stores, +1-3 % on the
        // 8B gate|up at T = 32768; neutral to -2 % on plain tiles, and -0.5 % in-engine where the
        // next GEMM could re-read the output from the caches (profiles/round4_ab_results.md)
        __builtin_amdgcn_raw_buffer_store_b128(o, rsC, (int)(vo + pr * 64), 0, SCH == 8 ? 2 : 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // the dummy pieces of the last K-tiles must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (DYN) {
    if (tid == 0) pf_retire(queue, P);
  }
}

namespace {
// one tile queue per (device, stream): launches on one stream run one after the other, so its
// heads are back at zero (reset by the last workgroup of the previous launch) when the next starts
int* pf_queue(hipStream_t s) {
  static std::mutex mu;
  static std::unordered_map<uint64_t, int*> queues;
  int dev = 0;
  DLLM_HIP_CHECK(hipGetDevice(&dev));
  const uint64_t key = ((uint64_t)(unsigned)dev << 56) ^ (uint64_t)(uintptr_t)s;
  std::lock_guard<std::mutex> g(mu);
  auto it = queues.find(key);
  if (it != queues.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  DLLM_HIP_CHECK(hipStreamIsCapturing(s, &cs));
  DLLM_HOST_CHECK(cs == hipStreamCaptureStatusNone, "gemm_pf's tile queue is created outside graph capture "
                                                    "(run the GEMM once on this stream before capturing)");
  int* q = nullptr;
  DLLM_HIP_CHECK(hipMalloc(&q, PF_QUEUE_INTS * sizeof(int)));
  DLLM_HIP_CHECK(hipMemsetAsync(q, 0, PF_QUEUE_INTS * sizeof(int), s));
  queues.emplace(key, q);
  return q;
}
}  // namespace

// Persistent prefill GEMM: C = A B^T (mode 0) or SwiGLU (mode 1, C [M, N / 2], B = [Bg; Bu]),
// 256 x 256 tiles, grid = min(tiles, CUs) rounded up to a multiple of 8.  variant bit 16: the
// dynamic tile queue (DYN; needs K >= 128) instead of the static tile = w + i P walk; variant 8:
// nontemporal output stores (by default: SwiGLU outputs > 256 MiB).
void gemm_pf(uintptr_t c, uintptr_t a, uintptr_t b, int M, int N, int K, int mode, int variant, uintptr_t stream) {
  const bool dyn = (variant & 16) != 0;
  variant &= ~16;
  DLLM_HOST_CHECK(!dyn || K >= 2 * PBK, "the dynamic tile queue needs K >= 128");
  DLLM_HOST_CHECK(M >= 1, "M >= 1");
  DLLM_HOST_CHECK(K % PBK == 0 && K >= PBK, "K must be a positive multiple of 64");
  DLLM_HOST_CHECK(N % 256 == 0, "N must be a multiple of 256");
  DLLM_HOST_CHECK(mode == 0 || mode == 1, "mode 0 (plain) or 1 (SwiGLU)");
  DLLM_HOST_CHECK(variant == 0 || variant == 8, "variant 0 or 8 (nontemporal output stores)");
  // the output's byte range must stay below 2^31: rows past M are dropped by giving their stores
  // the offset 0x80000000, which has to lie outside the buffer's range
  DLLM_HOST_CHECK((long)M * K * 2 < (1L << 32) && (long)N * K * 2 < (1L << 32) &&
                      (long)M * (mode == 1 ? N / 2 : N) * 2 < (1L << 31),
                  "operands must be < 4 GiB, the output < 2 GiB");
  // CUs of the current device, cached per device (a benign race: every thread stores the same value)
  static std::atomic<int> cus_of[64];
  int dev = 0;
  DLLM_HIP_CHECK(hipGetDevice(&dev));
  int cus = dev >= 0 && dev < 64 ? cus_of[dev].load(std::memory_order_relaxed) : 0;
  if (cus == 0) {
    int n = 0;
    DLLM_HIP_CHECK(hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev));
    cus = n > 0 ? n : 256;
    if (dev >= 0 && dev < 64) cus_of[dev].store(cus, std::memory_order_relaxed);
  }
  const long tiles = (long)(N / 256) * ((M + 255) / 256);
  DLLM_HOST_CHECK(tiles < (1L << 30), "tiles");
  const long grid = ((tiles < cus ? tiles : cus) + 7) / 8 * 8;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int* q = dyn ? pf_queue(s) : nullptr;
#define DLLM_PF_GO(MODE_, SCH_, DYN_)                                                                         \
  hipLaunchKernelGGL((gemm_pf_kernel<MODE_, SCH_, DYN_>), dim3((unsigned)grid), dim3(256), 0, s, (const bf16*)a, \
                     (const bf16*)b, (bf16*)c, M, N, K, q)
  const bool nt_store = variant == 8 || (mode == 1 && (long)M * (N / 2) * 2 > (256L << 20));
  if (mode == 1) {
    if (dyn) { if (nt_store) DLLM_PF_GO(2, 8, true); else DLLM_PF_GO(2, 0, true); }
    else { if (nt_store) DLLM_PF_GO(2, 8, false); else DLLM_PF_GO(2, 0, false); }
  } else {
    if (dyn) { if (nt_store) DLLM_PF_GO(0, 8, true); else DLLM_PF_GO(0, 0, true); }
    else { if (nt_store) DLLM_PF_GO(0, 8, false); else DLLM_PF_GO(0, 0, false); }
  }
#undef DLLM_PF_GO
  DLLM_HIP_CHECK(hipGetLastError());
}

}  // namespace dllm
