"""Stand-in for the native RCCL module (``_ext.rccl()``, csrc/comm/rccl_p2p.cpp) with the same
interface, for EXECUTING :class:`~.rccl_transport.RcclTransport`'s multi-rank code path where real
RCCL cannot run: several pipeline ranks on one GPU (RCCL refuses two ranks of one communicator on
one device; ``scripts/rccl_2rank_probe.py``, ``profiles/rccl_2rank_probe.txt``) or CPU-only hosts.
Selected with ``DLLM_RCCL_STANDIN=1`` (tests / rehearsal only; a warning is logged, and the bench
JSON reports the transport as ``rccl-standin``).

What runs is the transport's own logic -- the per-edge unique-id exchange over the control group,
the init order of the in-edge, out-edge and ring communicators, the three streams, the static
slot rings with their sent / consumed / landed events, the ids ring closure and abort -- with the
byte movement underneath replaced:

* ``unique_id()``: 128 random bytes (a real ncclUniqueId is 128 bytes too);
* ``RcclComm(nranks, rank, uid, device, timeout_s)``: a rendezvous on torch.distributed's default
  store under the uid (each member publishes its global rank, waits for the others');
* GPU ranks (``device >= 0``) -- DEVICE-ASYNCHRONOUS, like RCCL p2p: every rank owns an inbox per
  peer (a staging ring of ``SLOTS`` x ``CHUNK`` bytes plus flags, csrc/kernels/p2p_standin.hip) and
  exports it through HIP IPC; ``send`` / ``recv`` ENQUEUE a kernel on the caller's stream and
  return at once.  The send kernel writes chunks into the peer's inbox (spinning while the ring is
  full), the recv kernel spins on its CUs until each chunk has landed and copies it out -- so the
  hops occupy CUs and hardware queues and wait on the device, which is what the pipeline's
  scheduling has to survive with real RCCL (round-4 review: the host-synchronous stand-in hid it);
* CPU ranks (``device < 0``): bytes through the store under ``uid / src->dst / sequence`` keys,
  synchronously (host memory has no stream to wait on).
* ``abort()`` raises the host-mapped abort word every spinning kernel polls (they return within
  microseconds) and flags the communicator; later calls raise like the native one.  A kernel
  whose peer never shows up gives up at the deadline (``timeout_s``) and reports it in
  :meth:`RcclComm.status`.
"""
from __future__ import annotations

import ctypes
import datetime
import logging
import os
import time

import torch
import torch.distributed as dist

_hip = None


def _hiplib():
    global _hip
    if _hip is None:
        import glob
        cands = sorted(glob.glob(os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so*")))
        cands += ["libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"]
        last = None
        for c in cands:
            try:
                _hip = ctypes.CDLL(c)
                break
            except OSError as e:   # pragma: no cover - depends on the install
                last = e
        if _hip is None:           # pragma: no cover
            raise RuntimeError(f"rccl stand-in: libamdhip64 not loadable ({last})")
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
        _hip.hipSetDevice.argtypes = [ctypes.c_int]
    return _hip


_D2H, _H2D = 2, 1
log = logging.getLogger("dllm.rccl_standin")
_warned = False

# device inbox geometry: SLOTS chunks of CHUNK bytes in flight per edge, knobs.standin_channels
# workgroups per send / recv kernel (each moves a 1/channels piece of every chunk; RCCL's p2p
# channels), each holding knobs.standin_lds_kib of LDS (default 20 KiB, RCCL's own p2p kernel's
# 19,744 B on gfx950: a co-resident 144 KiB gemm_wide workgroup cannot share its CU)
CHUNK = 1 << 20
SLOTS = 4
CHANNELS = 4


def enabled() -> bool:
    return os.environ.get("DLLM_RCCL_STANDIN", "0") == "1"


def warn_selected():
    """Log once per process that the stand-in replaces RCCL (tests / rehearsal only)."""
    global _warned
    if not _warned:
        _warned = True
        log.warning("DLLM_RCCL_STANDIN=1: the RCCL transport runs over the stand-in communicators "
                    "(parallel/rccl_standin.py), not RCCL -- tests / one-GPU rehearsal only")


def _inject(stage: str):
    """Fault injection for the fallback tests: DLLM_RCCL_STANDIN_FAIL=<phase>:<global rank> makes
    that rank fail at <phase> ("uid": unique-id creation, "init": communicator construction)."""
    spec = os.environ.get("DLLM_RCCL_STANDIN_FAIL", "")
    if spec and dist.is_initialized():
        ph, _, r = spec.partition(":")
        if ph == stage and r and int(r) == dist.get_rank():
            raise RuntimeError(f"rccl stand-in: injected {stage} failure on rank {r}")


def unique_id() -> bytes:
    _inject("uid")
    return os.urandom(128)


def version() -> int:
    return 0


class RcclComm:
    def __init__(self, nranks: int, rank: int, uid: bytes, device: int, timeout_s: float = 0.0):
        if len(uid) != 128:
            raise ValueError("unique id must be 128 bytes")
        if not 0 <= rank < nranks:
            raise ValueError("rank out of range")
        if not dist.is_initialized():
            raise RuntimeError("rccl stand-in needs torch.distributed initialised (its store)")
        _inject("init")
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)
        self.timeout_s = float(timeout_s) if timeout_s and timeout_s > 0 else 600.0
        self._store = dist.distributed_c10d._get_default_store()
        self._key = "dllm_standin/" + uid[:16].hex()
        self._seq_tx = {}
        self._seq_rx = {}
        self._aborted = False
        if self.device >= 0:
            _hiplib().hipSetDevice(self.device)
        me = dist.get_rank()
        self._store.set(f"{self._key}/member/{self.rank}", str(me))
        self._peers = {}
        self._deadline_wait([f"{self._key}/member/{r}" for r in range(self.nranks)], "communicator init")
        for r in range(self.nranks):
            self._peers[r] = int(self._store.get(f"{self._key}/member/{r}"))
        from .. import knobs
        self._channels = max(1, int(knobs.K.standin_channels))   # both ends of an edge: one value
        self._words = None
        self._inbox = {}          # peer -> this rank's inbox tensor for messages FROM peer
        self._outbox = {}         # peer -> device pointer of the peer's inbox for messages from here
        self._mapped = []         # IPC bases to close on destroy
        if self.device >= 0:
            self._init_device()

    def _init_device(self):
        from .. import _ext
        k, m = _ext.kernels(), _ext.rccl_native()
        self._k = k
        self._words = k.p2p_host_words(2)             # [abort, error], coherent host memory
        self._wv = (ctypes.c_int * 2).from_address(self._words)
        dev = torch.device("cuda", self.device)
        nbytes = k.p2p_inbox_bytes(CHUNK, SLOTS)
        for p in range(self.nranks):
            if p == self.rank:
                continue
            buf = torch.zeros(nbytes, dtype=torch.uint8, device=dev)
            self._inbox[p] = buf
        torch.cuda.synchronize(dev)                   # zeroed flags before any peer maps them
        for p, buf in self._inbox.items():
            h, off = m.ipc_handle(buf.data_ptr())
            self._store.set(f"{self._key}/inbox/{p}->{self.rank}", bytes(h) + int(off).to_bytes(8, "little"))
        peers = [p for p in range(self.nranks) if p != self.rank]
        self._deadline_wait([f"{self._key}/inbox/{self.rank}->{p}" for p in peers], "inbox exchange")
        for p in peers:
            rec = self._store.get(f"{self._key}/inbox/{self.rank}->{p}")
            base, ptr = m.ipc_open(rec[:-8], int.from_bytes(rec[-8:], "little"), self.device)
            self._mapped.append(base)
            self._outbox[p] = ptr

    # ---- helpers
    def _deadline_wait(self, keys, what):
        t_end = time.monotonic() + self.timeout_s
        while True:
            if self._aborted:
                raise RuntimeError(f"RCCL {what}: communicator aborted")
            try:
                self._store.wait(keys, datetime.timedelta(seconds=1))
                return
            except Exception:   # noqa: BLE001 - store timeouts raise a generic error
                if time.monotonic() > t_end:
                    raise RuntimeError(f"RCCL {what}: peer did not respond within the timeout")

    def _live(self):
        if self._aborted:
            raise RuntimeError("RCCL communicator was aborted/destroyed")
        if self._words is not None and self._wv[1]:
            raise RuntimeError(f"RCCL stand-in: {self.status()}")

    def _launch(self, sptr, sbytes, speer, rptr, rbytes, rpeer, stream):
        """One device launch: a send to ``speer`` and / or a receive from ``rpeer`` (bytes 0 = none)."""
        s_inbox = r_inbox = 0
        s_seq = r_seq = 0
        if sbytes:
            s_inbox = self._outbox[speer]
            s_seq = self._seq_tx.get(speer, 0)
            self._seq_tx[speer] = s_seq + -(-int(sbytes) // CHUNK)
        if rbytes:
            r_inbox = self._inbox[rpeer].data_ptr()
            r_seq = self._seq_rx.get(rpeer, 0)
            self._seq_rx[rpeer] = r_seq + -(-int(rbytes) // CHUNK)
        from .. import knobs
        self._k.p2p_standin(int(sptr) if sbytes else 0, s_inbox, int(sbytes), s_seq, int(rptr) if rbytes else 0,
                            r_inbox, int(rbytes), r_seq, CHUNK, SLOTS, self._channels, self._words, self.timeout_s,
                            self._words + 4, knobs.K.standin_lds_kib << 10, int(stream))

    def _self_copy(self, dst, src, nbytes, stream):
        from .. import _ext
        _ext.rccl_native().copy_async(int(dst), int(src), int(nbytes), int(stream))

    def _sync(self, stream):
        if self.device >= 0 and stream:
            _hiplib().hipStreamSynchronize(ctypes.c_void_p(stream))
        elif self.device >= 0:
            torch.cuda.synchronize(self.device)

    def _read(self, ptr: int, nbytes: int) -> bytes:
        buf = ctypes.create_string_buffer(nbytes)
        if self.device >= 0:
            err = _hiplib().hipMemcpy(buf, ctypes.c_void_p(ptr), nbytes, _D2H)
            if err:
                raise RuntimeError(f"rccl stand-in: hipMemcpy D2H failed ({err})")
        else:
            ctypes.memmove(buf, ctypes.c_void_p(ptr), nbytes)
        return buf.raw

    def _write(self, ptr: int, data: bytes):
        if self.device >= 0:
            err = _hiplib().hipMemcpy(ctypes.c_void_p(ptr), data, len(data), _H2D)
            if err:
                raise RuntimeError(f"rccl stand-in: hipMemcpy H2D failed ({err})")
        else:
            ctypes.memmove(ctypes.c_void_p(ptr), data, len(data))

    # ---- the RcclComm interface
    def send(self, ptr: int, nbytes: int, peer: int, stream: int):
        self._live()
        if self.device >= 0:
            if peer == self.rank:
                raise RuntimeError("RCCL stand-in: a send to self must be grouped with its recv (sendrecv)")
            self._launch(ptr, nbytes, peer, 0, 0, -1, stream)
            return
        self._sync(stream)
        n = self._seq_tx.get(peer, 0)
        self._seq_tx[peer] = n + 1
        self._store.set(f"{self._key}/{self.rank}->{peer}/{n}", self._read(ptr, int(nbytes)))

    def recv(self, ptr: int, nbytes: int, peer: int, stream: int):
        self._live()
        if self.device >= 0:
            if peer == self.rank:
                raise RuntimeError("RCCL stand-in: a recv from self must be grouped with its send (sendrecv)")
            self._launch(0, 0, -1, ptr, nbytes, peer, stream)
            return
        self._sync(stream)
        n = self._seq_rx.get(peer, 0)
        self._seq_rx[peer] = n + 1
        key = f"{self._key}/{peer}->{self.rank}/{n}"
        self._deadline_wait([key], "recv")
        data = self._store.get(key)
        self._store.delete_key(key)
        if len(data) != int(nbytes):
            raise RuntimeError(f"rccl stand-in: received {len(data)} B, expected {nbytes} B")
        self._write(ptr, data)

    def sendrecv(self, sptr, sbytes, speer, rptr, rbytes, rpeer, stream):
        if self.device >= 0:
            self._live()
            if speer == self.rank and rpeer == self.rank:     # grouped self exchange: a device copy
                if sbytes != rbytes:
                    raise RuntimeError(f"RCCL stand-in: self exchange of {sbytes} B into {rbytes} B")
                self._self_copy(rptr, sptr, sbytes, stream)
                return
            self._launch(sptr, sbytes, speer, rptr, rbytes, rpeer, stream)
            return
        self.send(sptr, sbytes, speer, stream)
        self.recv(rptr, rbytes, rpeer, stream)

    def status(self) -> str:
        if self._words is not None and self._wv[1]:
            return {1: "aborted", 2: "RCCL stand-in: peer did not respond within the timeout"}.get(
                self._wv[1], f"RCCL stand-in: device error {self._wv[1]}")
        return "aborted" if self._aborted else ""

    def abort(self):
        """Every spinning kernel of this communicator returns (abort word); later calls raise."""
        self._aborted = True
        if self._words is not None:
            self._wv[0] = 1

    def destroy(self):
        """After the caller drained its streams: unmap the peers' inboxes.  An aborted communicator
        keeps its mappings (a kernel may still be leaving; the process is tearing down anyway)."""
        if self.device >= 0 and not self._aborted and self._mapped:
            from .. import _ext
            torch.cuda.synchronize(self.device)
            m = _ext.rccl_native()
            for base in self._mapped:
                m.ipc_close(base)
            self._mapped = []
        self._aborted = True

    @property
    def alive(self) -> bool:
        return not self._aborted
