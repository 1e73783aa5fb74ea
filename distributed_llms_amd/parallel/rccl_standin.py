"""Stand-in for the native RCCL module (``_ext.rccl()``, csrc/comm/rccl_p2p.cpp) with the same
interface, for EXECUTING :class:`~.rccl_transport.RcclTransport`'s multi-rank code path where real
RCCL cannot run: several pipeline ranks on one GPU (RCCL refuses two ranks of one communicator on
one device) or CPU-only hosts.  Selected with ``DLLM_RCCL_STANDIN=1`` (tests / rehearsal only).

What runs is the transport's own logic -- the per-edge unique-id exchange over the control group,
the init order of the in-edge, out-edge and ring communicators, the three streams, the static
slot rings with their sent / consumed / landed events, the ids ring closure and abort -- with only
the byte movement underneath replaced:

* ``unique_id()``: 128 random bytes (a real ncclUniqueId is 128 bytes too);
* ``RcclComm(nranks, rank, uid, device, timeout_s)``: a rendezvous on torch.distributed's default
  store under the uid (each member publishes its global rank, waits for the others');
* ``send`` / ``recv``: synchronise the caller's stream (the transport made it wait for the
  ready / consumed events), copy the bytes device -> host (hipMemcpy) or host memory directly,
  and hand them over through the store under ``uid / src->dst / sequence`` keys; the receiver
  copies host -> device before returning, so an event the transport records on the stream
  afterwards covers the landed bytes.  Host-synchronous -- a test vehicle, not a data plane.
* ``abort()`` flags the communicator; later calls raise like the native one.

``device < 0``: host-memory communicator (CPU stages).
"""
from __future__ import annotations

import ctypes
import datetime
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


def enabled() -> bool:
    return os.environ.get("DLLM_RCCL_STANDIN", "0") == "1"


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
        self._sync(stream)
        n = self._seq_tx.get(peer, 0)
        self._seq_tx[peer] = n + 1
        self._store.set(f"{self._key}/{self.rank}->{peer}/{n}", self._read(ptr, int(nbytes)))

    def recv(self, ptr: int, nbytes: int, peer: int, stream: int):
        self._live()
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
        self.send(sptr, sbytes, speer, stream)
        self.recv(rptr, rbytes, rpeer, stream)

    def status(self) -> str:
        return "aborted" if self._aborted else ""

    def abort(self):
        self._aborted = True

    def destroy(self):
        self._aborted = True

    @property
    def alive(self) -> bool:
        return not self._aborted
