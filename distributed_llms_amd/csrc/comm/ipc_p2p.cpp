// N6: HIP-IPC peer-write data plane for pipeline hops.
//
// A receiving stage exports a ring of activation slots and a flag word per slot
// (hipIpcGetMemHandle); the sending stage maps them (hipIpcOpenMemHandle) and, on its comm
// stream, copies the microbatch straight into the receiver's HBM over xGMI (same-device IPC on a
// 1-GPU box) and then raises the slot's flag with hipStreamWriteValue32.  The receiver's compute
// stream waits for the flag in the command processor (hipStreamWaitValue32: no wave spins, no host
// thread blocks) and hands the credit back the same way once the slot's consumers are queued.
// No RCCL kernel launch or proxy thread sits between two stages: a hop is one copy + two
// stream memory operations.
//
// Handles are the BASE of the allocation (what hipIpcGetMemHandle maps); a torch tensor inside
// the caching allocator's block carries its offset from hipMemGetAddressRange.
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

void ipc_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// (handle bytes, byte offset of ptr inside its allocation)
py::tuple ipc_handle(uintptr_t ptr) {
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  ipc_check(hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(ptr)), "hipMemGetAddressRange");
  hipIpcMemHandle_t h;
  ipc_check(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(base)), "hipIpcGetMemHandle");
  const uintptr_t off = ptr - reinterpret_cast<uintptr_t>(base);
  return py::make_tuple(py::bytes(h.reserved, HIP_IPC_HANDLE_SIZE), off);
}

// maps a peer's exported allocation; returns (base, base + offset)
py::tuple ipc_open(const std::string& handle, uintptr_t offset, int device) {
  if (handle.size() != HIP_IPC_HANDLE_SIZE) throw std::invalid_argument("IPC handle must be 64 bytes");
  hipIpcMemHandle_t h;
  std::memcpy(h.reserved, handle.data(), HIP_IPC_HANDLE_SIZE);
  ipc_check(hipSetDevice(device), "hipSetDevice");
  void* p = nullptr;
  ipc_check(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess), "hipIpcOpenMemHandle");
  const uintptr_t base = reinterpret_cast<uintptr_t>(p);
  return py::make_tuple(base, base + offset);
}

void ipc_close(uintptr_t base) { ipc_check(hipIpcCloseMemHandle(reinterpret_cast<void*>(base)), "hipIpcCloseMemHandle"); }

void copy_async(uintptr_t dst, uintptr_t src, long nbytes, uintptr_t stream) {
  if (nbytes <= 0) return;
  ipc_check(hipMemcpyAsync(reinterpret_cast<void*>(dst), reinterpret_cast<const void*>(src), (size_t)nbytes,
                           hipMemcpyDeviceToDevice, reinterpret_cast<hipStream_t>(stream)),
            "hipMemcpyAsync");
}

void write_value32(uintptr_t stream, uintptr_t ptr, uint32_t value) {
  ipc_check(hipStreamWriteValue32(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<void*>(ptr), value, 0),
            "hipStreamWriteValue32");
}

// the stream proceeds once *ptr >= value (unsigned)
void wait_value32(uintptr_t stream, uintptr_t ptr, uint32_t value) {
  ipc_check(hipStreamWaitValue32(reinterpret_cast<hipStream_t>(stream), reinterpret_cast<void*>(ptr), value,
                                 hipStreamWaitValueGte, 0xFFFFFFFFu),
            "hipStreamWaitValue32");
}

// A stream with a CU mask.  HIP never pools such a stream with others on a shared hardware queue
// (the mask is a queue property), so a communication kernel that spins on it -- an RCCL receive
// posted before its peer sends -- cannot hold up the compute stream's kernels behind it in one
// in-order queue (a process gets GPU_MAX_HW_QUEUES = 4 hardware queues; streams beyond that share).
// mask: one bit per CU, 32 CUs per word; an empty list = every CU.
uintptr_t cu_masked_stream(int device, const std::vector<uint32_t>& mask) {
  ipc_check(hipSetDevice(device), "hipSetDevice");
  std::vector<uint32_t> m(mask);
  if (m.empty()) {
    int cus = 0;
    ipc_check(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device), "hipDeviceGetAttribute");
    m.assign((cus + 31) / 32, 0u);
    for (int c = 0; c < cus; ++c) m[c / 32] |= 1u << (c % 32);
  }
  hipStream_t st = nullptr;
  ipc_check(hipExtStreamCreateWithCUMask(&st, (uint32_t)m.size(), m.data()), "hipExtStreamCreateWithCUMask");
  return reinterpret_cast<uintptr_t>(st);
}

// A non-blocking stream at the device's greatest priority.  HIP gives high-priority streams their
// own pool of hardware queues (up to GPU_MAX_HW_QUEUES, then shared): the first few such streams of
// a process each get a queue no normal-priority stream uses (profiles/round5_comm_queues.md).
uintptr_t priority_stream(int device) {
  ipc_check(hipSetDevice(device), "hipSetDevice");
  int least = 0, greatest = 0;
  ipc_check(hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
  hipStream_t st = nullptr;
  ipc_check(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest), "hipStreamCreateWithPriority");
  return reinterpret_cast<uintptr_t>(st);
}

// A non-blocking stream at normal priority, owned by the caller (not torch's stream pool, which hands
// its 32 streams out round-robin: a pool stream probed onto a queue of its own could later be handed
// to another user and put that user's work behind a spinning receive).
uintptr_t plain_stream(int device) {
  ipc_check(hipSetDevice(device), "hipSetDevice");
  hipStream_t st = nullptr;
  ipc_check(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreateWithFlags");
  return reinterpret_cast<uintptr_t>(st);
}

void stream_destroy(uintptr_t st) { ipc_check(hipStreamDestroy(reinterpret_cast<hipStream_t>(st)), "hipStreamDestroy"); }

bool can_wait_value(int device) {
  int v = 0;
  ipc_check(hipDeviceGetAttribute(&v, hipDeviceAttributeCanUseStreamWaitValue, device), "hipDeviceGetAttribute");
  return v != 0;
}

}  // namespace

void register_ipc(py::module_& m) {
  m.def("ipc_handle", &ipc_handle, py::arg("ptr"), "(64-byte IPC handle of ptr's allocation, offset of ptr in it)");
  m.def("ipc_open", &ipc_open, py::arg("handle"), py::arg("offset"), py::arg("device"),
        "map a peer allocation: (base, base + offset)");
  m.def("ipc_close", &ipc_close, py::arg("base"));
  m.def("copy_async", &copy_async, py::arg("dst"), py::arg("src"), py::arg("nbytes"), py::arg("stream"));
  m.def("write_value32", &write_value32, py::arg("stream"), py::arg("ptr"), py::arg("value"));
  m.def("wait_value32", &wait_value32, py::arg("stream"), py::arg("ptr"), py::arg("value"));
  m.def("can_wait_value", &can_wait_value, py::arg("device"));
  m.def("cu_masked_stream", &cu_masked_stream, py::arg("device"), py::arg("mask") = std::vector<uint32_t>{},
        "a HIP stream on a hardware queue of its own (CU mask; empty = all CUs)");
  m.def("priority_stream", &priority_stream, py::arg("device"),
        "a non-blocking stream at the greatest priority (a hardware queue of its own, up to the queue limit)");
  m.def("plain_stream", &plain_stream, py::arg("device"),
        "a non-blocking normal-priority stream owned by the caller (outside torch's stream pool)");
  m.def("stream_destroy", &stream_destroy, py::arg("stream"));
}
