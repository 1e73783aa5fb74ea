// N3: native RCCL point-to-point transport for pipeline activations.
//
// One communicator per pipeline (rank = stage index), created from a unique id that stage 0
// generates and the control plane distributes.  send/recv are ncclSend/ncclRecv of raw bytes
// on a caller-chosen HIP stream -- the pipeline runs them on a dedicated comm stream ordered
// against the compute stream with HIP events, so a stage's next microbatch never waits behind
// a transfer, and (because RCCL p2p is graph-capturable) a stage step can later be captured
// together with its hops.  abort() is ncclCommAbort: pending transfers against a dead peer
// return instead of hanging (membership change).
//
// Links against the librccl.so that PyTorch already loaded (same SONAME), so the process keeps
// ONE RCCL instance; the header comes from /opt/rocm/include/rccl.
#include <hip/hip_runtime_api.h>
#include <pybind11/pybind11.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <mutex>
#include <cstring>
#include <stdexcept>
#include <string>
#include <thread>

namespace py = pybind11;

namespace {

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess && r != ncclInProgress)
    throw std::runtime_error(std::string("RCCL ") + what + " failed: " + ncclGetErrorString(r));
}

void hip_check(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

py::bytes unique_id() {
  ncclUniqueId id;
  check(ncclGetUniqueId(&id), "ncclGetUniqueId");
  return py::bytes(id.internal, NCCL_UNIQUE_ID_BYTES);
}

class RcclComm {
 public:
  // timeout_s > 0: a NON-BLOCKING communicator -- init and every enqueue that returns
  // ncclInProgress (lazy p2p connection setup) are polled against the deadline, and a peer that
  // never shows up aborts the communicator and raises instead of hanging the rank forever.
  //
  // Threading: send / recv / sendrecv release the GIL for the whole enqueue + settle (the first
  // hop of an edge can wait seconds for its peer: the heartbeat thread, the master handler and
  // the teardown path must keep running meanwhile).  mu_ serialises the calls that use comm_;
  // abort() first raises aborting_ -- every settle loop and every later call sees it and leaves
  // without touching comm_ -- then takes mu_ (bounded wait) and aborts, so a serve thread still
  // inside a send can never use a communicator abort() has freed.
  RcclComm(int nranks, int rank, const std::string& uid, int device, double timeout_s)
      : nranks_(nranks), rank_(rank), timeout_s_(timeout_s) {
    if (uid.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("unique id must be 128 bytes");
    if (rank < 0 || rank >= nranks) throw std::invalid_argument("rank out of range");
    ncclUniqueId id;
    std::memcpy(id.internal, uid.data(), NCCL_UNIQUE_ID_BYTES);
    hip_check(hipSetDevice(device), "hipSetDevice");
    py::gil_scoped_release nogil;   // init rendezvous blocks until every rank joins
    std::lock_guard<std::timed_mutex> g(mu_);
    if (timeout_s_ > 0) {
      ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
      cfg.blocking = 0;
      check(ncclCommInitRankConfig(&comm_, nranks, id, rank, &cfg), "ncclCommInitRankConfig");
      settle("ncclCommInitRank");
    } else {
      check(ncclCommInitRank(&comm_, nranks, id, rank), "ncclCommInitRank");
    }
  }
  ~RcclComm() {
    if (comm_) ncclCommDestroy(comm_);
  }

  void send(uintptr_t ptr, long nbytes, int peer, uintptr_t stream) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::timed_mutex> g(mu_);
    live();
    enqueue(ncclSend(reinterpret_cast<const void*>(ptr), (size_t)nbytes, ncclUint8, peer, comm_,
                     reinterpret_cast<hipStream_t>(stream)), "ncclSend");
  }
  void recv(uintptr_t ptr, long nbytes, int peer, uintptr_t stream) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::timed_mutex> g(mu_);
    live();
    enqueue(ncclRecv(reinterpret_cast<void*>(ptr), (size_t)nbytes, ncclUint8, peer, comm_,
                     reinterpret_cast<hipStream_t>(stream)), "ncclRecv");
  }
  // fused exchange (both directions in one group: no ordering deadlock between the two; also the
  // only legal form of a send to self)
  void sendrecv(uintptr_t sptr, long sbytes, int speer, uintptr_t rptr, long rbytes, int rpeer, uintptr_t stream) {
    py::gil_scoped_release nogil;
    std::lock_guard<std::timed_mutex> g(mu_);
    live();
    check(ncclGroupStart(), "ncclGroupStart");
    check(ncclSend(reinterpret_cast<const void*>(sptr), (size_t)sbytes, ncclUint8, speer, comm_,
                   reinterpret_cast<hipStream_t>(stream)), "ncclSend");
    check(ncclRecv(reinterpret_cast<void*>(rptr), (size_t)rbytes, ncclUint8, rpeer, comm_,
                   reinterpret_cast<hipStream_t>(stream)), "ncclRecv");
    enqueue(ncclGroupEnd(), "ncclGroupEnd");
  }
  // the communicator's asynchronous error state: "" (healthy), "in_progress", or the error text
  std::string status() {
    if (aborting_.load()) return "aborted";
    std::unique_lock<std::timed_mutex> g(mu_, std::try_to_lock);
    if (!g.owns_lock()) return "in_progress";   // a call is settling right now
    if (!comm_) return "aborted";
    ncclResult_t r = ncclSuccess;
    ncclCommGetAsyncError(comm_, &r);
    if (r == ncclSuccess) return "";
    if (r == ncclInProgress) return "in_progress";
    return ncclGetErrorString(r);
  }
  void abort() {
    aborting_.store(true);
    py::gil_scoped_release nogil;
    // a settling call notices aborting_ within one poll (50 us); a call blocked INSIDE RCCL (a
    // blocking communicator's lazy connect) never returns on its own: after the bounded wait the
    // abort goes ahead without the lock -- that call then finds aborting_ set and leaves without
    // touching comm_
    std::unique_lock<std::timed_mutex> g(mu_, std::defer_lock);
    (void)g.try_lock_for(std::chrono::seconds(2));
    ncclComm_t c = comm_;
    comm_ = nullptr;
    if (c) ncclCommAbort(c);
  }
  void destroy() {
    py::gil_scoped_release nogil;
    std::lock_guard<std::timed_mutex> g(mu_);
    if (comm_) {
      ncclComm_t c = comm_;
      comm_ = nullptr;
      check(ncclCommDestroy(c), "ncclCommDestroy");
    }
  }
  int rank() const { return rank_; }
  int nranks() const { return nranks_; }
  bool alive() const { return comm_ != nullptr && !aborting_.load(); }

 private:
  void live() const {
    if (!comm_ || aborting_.load()) throw std::runtime_error("RCCL communicator was aborted/destroyed");
  }
  void enqueue(ncclResult_t r, const char* what) {
    if (aborting_.load()) throw std::runtime_error(std::string("RCCL ") + what + ": communicator aborted");
    check(r, what);
    if (r == ncclInProgress || timeout_s_ > 0) settle(what);
  }
  // poll a non-blocking communicator until its last call finished; abort + raise at the deadline.
  // Caller holds mu_.
  void settle(const char* what) {
    if (timeout_s_ <= 0) return;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s_);
    for (;;) {
      if (aborting_.load()) throw std::runtime_error(std::string("RCCL ") + what + ": communicator aborted");
      ncclResult_t r = ncclSuccess;
      ncclCommGetAsyncError(comm_, &r);
      if (r == ncclSuccess) return;
      if (r != ncclInProgress || std::chrono::steady_clock::now() > t_end) {
        aborting_.store(true);
        ncclComm_t c = comm_;
        comm_ = nullptr;
        ncclCommAbort(c);
        throw std::runtime_error(std::string("RCCL ") + what +
                                 (r != ncclInProgress ? std::string(" failed: ") + ncclGetErrorString(r)
                                                      : std::string(": peer did not respond within the timeout")));
      }
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
  ncclComm_t comm_ = nullptr;
  int nranks_, rank_;
  double timeout_s_;
  std::timed_mutex mu_;
  std::atomic<bool> aborting_{false};
};

}  // namespace

void register_ipc(py::module_& m);   // ipc_p2p.cpp (N6)

PYBIND11_MODULE(_C_rccl, m) {
  m.doc() = "Native RCCL p2p transport and HIP-IPC peer-write data plane (pipeline activations over xGMI)";
  register_ipc(m);
  m.def("unique_id", &unique_id);
  m.def("version", []() {
    int v = 0;
    ncclGetVersion(&v);
    return v;
  });
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init<int, int, const std::string&, int, double>(), py::arg("nranks"), py::arg("rank"), py::arg("uid"),
           py::arg("device"), py::arg("timeout_s") = 0.0)
      .def("send", &RcclComm::send, py::arg("ptr"), py::arg("nbytes"), py::arg("peer"), py::arg("stream"))
      .def("recv", &RcclComm::recv, py::arg("ptr"), py::arg("nbytes"), py::arg("peer"), py::arg("stream"))
      .def("sendrecv", &RcclComm::sendrecv)
      .def("abort", &RcclComm::abort)
      .def("status", &RcclComm::status)
      .def("destroy", &RcclComm::destroy)
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("nranks", &RcclComm::nranks)
      .def_property_readonly("alive", &RcclComm::alive);
}
