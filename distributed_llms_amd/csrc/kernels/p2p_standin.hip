// Device-side stand-in for RCCL point-to-point send / recv (parallel/rccl_standin.py).
//
// Real RCCL refuses two ranks of one communicator on one device, so the multi-rank pipeline
// rehearsal on a one-GPU box needs a stand-in.  This one keeps what matters for the pipeline's
// scheduling on the GPU -- it is NOT host-synchronous:
//   * ncclSend / ncclRecv are kernels enqueued on the caller's stream; they occupy CUs (one
//     256-thread workgroup per "channel") and sit in the stream's hardware queue;
//   * a recv kernel SPINS on its CU until the peer's send kernel has written the bytes, and a send
//     kernel spins until the receiver has drained a staging slot, exactly like RCCL's simple
//     protocol (a bounded FIFO of slots per connection, flags in device memory).
//
// Layout: the RECEIVER owns one inbox per (sender -> receiver) edge, a single device allocation
// that the sender maps through HIP IPC (same device: the same HBM and the same L2s):
//
//   [nslots x chunk bytes of staging][full flag per (slot, channel)][consumed counter per channel]
//
// every flag on a 128-byte line of its own.  Chunk s of the edge (a running sequence number over
// all messages, kept by the host) goes to slot s % nslots; channel w of both kernels moves bytes
// [w * piece, (w + 1) * piece) of every chunk, so the channels never wait for one another.
//   sender, channel w:   wait consumed[w] >= s + 1 - nslots  (the slot's previous chunk is read)
//                        copy its piece into the slot
//                        every wave: vmcnt(0); barrier; lane 0: release (agent); vmcnt(0);
//                        full[slot][w] = s + 1
//   receiver, channel w: wait full[slot][w] >= s + 1; acquire (agent); vmcnt(0); barrier
//                        copy its piece out of the slot into the destination
//                        vmcnt(0) (the loads have returned); barrier; consumed[w] = s + 1
// (the hand-off recipe of the MI355X guide: plain stores + agent release before a relaxed flag
// store; one relaxed poll, then one agent acquire before plain loads).  Every spin has an exit
// condition every wave reaches: the host's abort word (pinned host memory) or a wall-clock
// deadline (s_memrealtime, 100 MHz); the kernel then records an error code and returns.
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "common.h"
#include "launchers.h"

namespace dllm {
namespace {

constexpr int kP2pThreads = 256;
constexpr int kMaxChannels = 16;
constexpr int kFlagStride = 16;        // u64 per flag line (128 B)

struct P2pRole {
  const uint8_t* src;      // send: message source      recv: inbox staging base
  uint8_t* dst;            // send: peer inbox staging  recv: message destination
  uint64_t* full;          // [nslots][kMaxChannels] * kFlagStride
  uint64_t* consumed;      // [kMaxChannels] * kFlagStride
  long nbytes;
  long chunk;
  int nslots;
  int channels;
  uint64_t seq0;
};

__device__ __forceinline__ uint64_t ld_relaxed(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_relaxed(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// lane 0 of the workgroup spins until *flag >= want; 0 on success, else an error code
// (1: aborted by the host, 2: deadline).  The verdict goes to every thread through LDS.
__device__ int spin_until(const uint64_t* flag, uint64_t want, const int* abort_word, uint64_t deadline,
                          int* verdict) {
  if (threadIdx.x == 0) {
    int v = 0;
    uint32_t n = 0;
    while (ld_relaxed(flag) < want) {
      if ((++n & 255) == 0) {
        if (abort_word != nullptr && __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
          v = 1;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() > deadline) {
          v = 2;
          break;
        }
      }
      __builtin_amdgcn_s_sleep(2);
    }
    *verdict = v;
  }
  __syncthreads();
  return *verdict;
}

// copy [0, n) bytes: 16-byte vectors, 4 in flight per thread, when both ends are 16-byte aligned
// (activation hops always are); bytes otherwise (small unaligned id vectors)
__device__ __forceinline__ void copy_piece(uint8_t* __restrict__ d, const uint8_t* __restrict__ s, long n) {
  if (((reinterpret_cast<uintptr_t>(d) | reinterpret_cast<uintptr_t>(s)) & 15) != 0) {
    for (long j = threadIdx.x; j < n; j += kP2pThreads) d[j] = s[j];
    return;
  }
  const long nv = n >> 4;
  const uint4* sv = reinterpret_cast<const uint4*>(s);
  uint4* dv = reinterpret_cast<uint4*>(d);
  long i = threadIdx.x;
  for (; i + 3 * kP2pThreads < nv; i += 4 * kP2pThreads) {
    const uint4 a = sv[i], b = sv[i + kP2pThreads], c = sv[i + 2 * kP2pThreads], e = sv[i + 3 * kP2pThreads];
    dv[i] = a;
    dv[i + kP2pThreads] = b;
    dv[i + 2 * kP2pThreads] = c;
    dv[i + 3 * kP2pThreads] = e;
  }
  for (; i < nv; i += kP2pThreads) dv[i] = sv[i];
  for (long j = (nv << 4) + threadIdx.x; j < n; j += kP2pThreads) d[j] = s[j];
}

__device__ __forceinline__ void report(int* err, int v) {
  if (threadIdx.x == 0) __hip_atomic_store(err, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ void run_send(const P2pRole& r, int w, const int* abort_word, uint64_t deadline, int* err,
                         int* verdict) {
  const long nchunks = (r.nbytes + r.chunk - 1) / r.chunk;
  const long piece = ((r.chunk / r.channels) + 15) & ~15L;
  for (long c = 0; c < nchunks; ++c) {
    const uint64_t s = r.seq0 + (uint64_t)c;
    const int slot = (int)(s % (uint64_t)r.nslots);
    const long len = min(r.chunk, r.nbytes - c * r.chunk);
    const long a = min(len, (long)w * piece), b = min(len, (long)(w + 1) * piece);
    if (s + 1 > (uint64_t)r.nslots) {
      const int v = spin_until(r.consumed + w * kFlagStride, s + 1 - r.nslots, abort_word, deadline, verdict);
      if (v) {
        report(err, v);
        return;
      }
    }
    if (b > a) copy_piece(r.dst + (long)slot * r.chunk + a, r.src + c * r.chunk + a, b - a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_relaxed(r.full + ((long)slot * kMaxChannels + w) * kFlagStride, s + 1);
    }
  }
}

__device__ void run_recv(const P2pRole& r, int w, const int* abort_word, uint64_t deadline, int* err,
                         int* verdict) {
  const long nchunks = (r.nbytes + r.chunk - 1) / r.chunk;
  const long piece = ((r.chunk / r.channels) + 15) & ~15L;
  for (long c = 0; c < nchunks; ++c) {
    const uint64_t s = r.seq0 + (uint64_t)c;
    const int slot = (int)(s % (uint64_t)r.nslots);
    const long len = min(r.chunk, r.nbytes - c * r.chunk);
    const long a = min(len, (long)w * piece), b = min(len, (long)(w + 1) * piece);
    const int v = spin_until(r.full + ((long)slot * kMaxChannels + w) * kFlagStride, s + 1, abort_word, deadline,
                             verdict);
    if (v) {
      report(err, v);
      return;
    }
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (b > a) copy_piece(r.dst + c * r.chunk + a, r.src + (long)slot * r.chunk + a, b - a);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) st_relaxed(r.consumed + w * kFlagStride, s + 1);
  }
}

// blocks [0, send.channels) send, the rest receive (a grouped send + recv is one launch, so the two
// halves of an exchange on one stream cannot wait on each other)
__global__ void __launch_bounds__(kP2pThreads) p2p_standin_kernel(P2pRole send, P2pRole recv,
                                                                   const int* abort_word, uint64_t timeout_ticks,
                                                                   int* err) {
  __shared__ int verdict;
  const int b = blockIdx.x;
  const uint64_t deadline = __builtin_amdgcn_s_memrealtime() + timeout_ticks;   // 100 MHz clock
  if (b < send.channels)
    run_send(send, b, abort_word, deadline, err, &verdict);
  else
    run_recv(recv, b - send.channels, abort_word, deadline, err, &verdict);
}

P2pRole make_role(uintptr_t src, uintptr_t dst, uintptr_t inbox, long nbytes, long chunk, int nslots, int channels,
                  uint64_t seq0) {
  P2pRole r{};
  if (nbytes <= 0) return r;
  uint8_t* base = reinterpret_cast<uint8_t*>(inbox);
  r.src = reinterpret_cast<const uint8_t*>(src);
  r.dst = reinterpret_cast<uint8_t*>(dst);
  r.full = reinterpret_cast<uint64_t*>(base + (long)nslots * chunk);
  r.consumed = r.full + (long)nslots * kMaxChannels * kFlagStride;
  r.nbytes = nbytes;
  r.chunk = chunk;
  r.nslots = nslots;
  r.channels = channels;
  r.seq0 = seq0;
  return r;
}

}  // namespace

long p2p_inbox_bytes(long chunk, int nslots) {
  return (long)nslots * chunk + ((long)nslots * kMaxChannels + kMaxChannels) * kFlagStride * 8;
}

// One launch moving a send and / or a receive of raw bytes through an edge inbox.
//   send: src (this rank's message) -> s_inbox (the PEER's inbox for this rank, IPC-mapped)
//   recv: r_inbox (this rank's inbox for the peer) -> dst
// seq0: the edge's chunk counter before this message (the host advances it by ceil(nbytes/chunk)).
// lds_bytes: LDS each channel workgroup reserves (untouched) -- a communication kernel's footprint
// decides whether a co-resident persistent GEMM's workgroup still fits on its CU.
void p2p_standin(uintptr_t src, uintptr_t s_inbox, long s_bytes, uint64_t s_seq0, uintptr_t dst, uintptr_t r_inbox,
                 long r_bytes, uint64_t r_seq0, long chunk, int nslots, int channels, uintptr_t abort_word,
                 double timeout_s, uintptr_t err, int lds_bytes, uintptr_t stream) {
  DLLM_HOST_CHECK(lds_bytes >= 0 && lds_bytes <= 64 * 1024, "p2p LDS reservation in [0, 64 KiB]");
  DLLM_HOST_CHECK(chunk > 0 && chunk % (16L * 64) == 0, "p2p chunk must be a positive multiple of 1 KiB");
  DLLM_HOST_CHECK(nslots >= 2 && nslots <= 64, "p2p slots in [2, 64]");
  DLLM_HOST_CHECK(channels >= 1 && channels <= kMaxChannels, "p2p channels in [1, 16]");
  DLLM_HOST_CHECK(chunk / channels >= 16, "p2p chunk too small for its channels");
  DLLM_HOST_CHECK(s_bytes >= 0 && r_bytes >= 0, "p2p message sizes");
  DLLM_HOST_CHECK(s_bytes == 0 || (src && s_inbox), "p2p send needs a source and the peer inbox");
  DLLM_HOST_CHECK(r_bytes == 0 || (dst && r_inbox), "p2p recv needs a destination and an inbox");
  DLLM_HOST_CHECK(err != 0 && abort_word != 0, "p2p error / abort words (p2p_host_words)");
  if (s_bytes == 0 && r_bytes == 0) return;
  P2pRole s = make_role(src, s_inbox, s_inbox, s_bytes, chunk, nslots, channels, s_seq0);
  P2pRole r = make_role(r_inbox, dst, r_inbox, r_bytes, chunk, nslots, channels, r_seq0);
  s.channels = s_bytes ? channels : 0;
  r.channels = r_bytes ? channels : 0;
  // the deadline counts from the kernel's start: a kernel queued behind a long stream prefix does
  // not time out before it even runs
  const uint64_t ticks = (uint64_t)((timeout_s > 0 ? timeout_s : 600.0) * 1e8);
  const int grid = s.channels + r.channels;
  hipLaunchKernelGGL(p2p_standin_kernel, dim3(grid), dim3(kP2pThreads), (unsigned)lds_bytes,
                     reinterpret_cast<hipStream_t>(stream),
                     s, r, reinterpret_cast<const int*>(abort_word), ticks, reinterpret_cast<int*>(err));
  DLLM_HIP_CHECK(hipGetLastError());
}

// Coherent, device-mapped host words: [0] the abort flag the host raises, [1] the error code a
// kernel reports (1: aborted, 2: deadline).  The host reads and writes them without a sync.
uintptr_t p2p_host_words(int n) {
  DLLM_HOST_CHECK(n > 0 && n <= 4096, "p2p host words");
  void* p = nullptr;
  DLLM_HIP_CHECK(hipHostMalloc(&p, sizeof(int) * (size_t)n, hipHostMallocCoherent | hipHostMallocMapped));
  for (int i = 0; i < n; ++i) static_cast<volatile int*>(p)[i] = 0;
  return reinterpret_cast<uintptr_t>(p);
}

void p2p_host_words_free(uintptr_t p) {
  if (p) DLLM_HIP_CHECK(hipHostFree(reinterpret_cast<void*>(p)));
}

}  // namespace dllm
