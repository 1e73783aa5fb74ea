"""Pipeline transports: the data plane between stages.

Three message kinds flow along a pipeline:
  meta    stage s -> s+1   packed int32 HostBatch (block tables, slots, ...)   CPU, control group
  hidden  stage s -> s+1   [T, H] bf16 activations                            device, data group
  ids     last  -> stage 0 sampled ids [B] int32 (ring closure)              device, ring group

``DistTransport`` rides on torch.distributed: activations on the default group (backend
"nccl" = RCCL over xGMI on MI355X, gloo on CPU) as point-to-point isend/recv, whose
launches torch orders against the compute stream with events; control messages on a
separate gloo group so they never serialise behind GPU work.  The ring closure has a group of
its own ({stage 0, last stage}): a communicator -- and an RCCL stream -- separate from the
activation pair's, so at pp = 2, where both flows join the same two ranks, a posted ids receive
never queues an activation send behind it (p2p ops of one communicator are stream-ordered).
Stage 0 posts each microbatch's ids receive when it issues the microbatch, feeds the device
ids straight into the slot's next decode step (lookahead) and reads them on the host one step
later for bookkeeping -- the host is not on the ring's critical path.  ``LoopbackTransport`` is
the same interface over in-process queues, so N stage threads can share one GPU
(NCCL-family libraries refuse two ranks of one communicator on one device) -- this is
how the pipeline schedule is exercised on the single-GPU test box.
"""
from __future__ import annotations

import functools
import queue
import threading
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

STOP = -1


def sync_event(ev, timeout_s: float, what: str = "pipeline peer"):
    """ev.synchronize() with a deadline: a dead pipeline peer must not hang the host forever."""
    if ev.query():
        return
    import time
    t_end = time.monotonic() + timeout_s
    delay = 2e-5
    while not ev.query():
        if time.monotonic() > t_end:
            raise TimeoutError(f"{what}: no data after {timeout_s:.0f} s (peer dead or hung)")
        time.sleep(delay)
        delay = min(delay * 2, 1e-3)


class PendingIds:
    """One microbatch's sampled ids on their way from the last stage to stage 0.

    ``wait()`` returns the ids tensor once it may be used: on a GPU stage it orders the CURRENT
    stream after the arrival (no host block); on CPU it blocks.  ``host()`` returns them as numpy
    (blocking); with a ``copy_stream`` the device -> pinned copy is queued at post time so the
    host read later finds it done.

    ``post``: a DEFERRED device receive (RCCL transport).  Nothing is enqueued until the ids are
    first needed: ``wait()`` runs ``post()`` on the current stream -- the receive lands right in
    front of its consumer -- and queues the device -> pinned copy behind it; ``host()`` does the same
    and blocks.  A receive posted early on a stream of its own spins in that stream's hardware
    queue for a whole pipeline cycle, and HIP shares queues between streams: whatever compute
    shares it stalls until the ids arrive (pp2 over the device stand-in: stage 0 busy 69 %,
    76 % of the IPC rehearsal; profiles/round5_pp_rehearsal.md)."""

    def __init__(self, tensor: Optional[torch.Tensor] = None, work=None, ready=None, fetch=None,
                 copy_stream=None, timeout_s: float = 600.0, post=None):
        self.tensor = tensor
        self.timeout_s = timeout_s
        self._work = work          # torch.distributed Work (NCCL: stream-orders; gloo: blocks)
        self._ready = ready        # torch.cuda.Event recorded when `tensor` was filled
        self._fetch = fetch        # loopback: blocking getter -> (tensor, event or None)
        self._post = post          # deferred device receive: enqueue on the current stream
        self._host = None
        self._host_ev = None
        self._foreign = False
        if copy_stream is not None and tensor is not None and tensor.is_cuda:
            with torch.cuda.stream(copy_stream):
                self.wait()
                self._host = torch.empty(tensor.shape, dtype=tensor.dtype).pin_memory()
                self._host.copy_(tensor, non_blocking=True)
                self._host_ev = torch.cuda.Event()
                self._host_ev.record(copy_stream)

    @property
    def posted(self) -> bool:
        return self._post is None

    def post(self):
        """Enqueue the deferred receive (and the host copy behind it) on the current stream."""
        if self._post is None:
            return
        post, self._post = self._post, None
        post()
        cur = torch.cuda.current_stream()
        self._host = torch.empty(self.tensor.shape, dtype=self.tensor.dtype).pin_memory()
        self._host.copy_(self.tensor, non_blocking=True)
        self._host_ev = torch.cuda.Event()
        self._host_ev.record(cur)

    def wait(self) -> torch.Tensor:
        if self._post is not None:
            self.post()                # stream-ordered: the receive precedes its consumers
            return self.tensor
        if self._fetch is not None:
            self.tensor, self._ready = self._fetch()
            self._fetch = None
            self._foreign = self.tensor.is_cuda and self._ready is not None   # another thread's stream
        if self._work is not None:
            self._work.wait()
            if not (self.tensor is not None and self.tensor.is_cuda):
                self._work = None     # CPU: done once
        if self._ready is not None:
            cur = torch.cuda.current_stream()
            cur.wait_event(self._ready)
            if self._foreign:
                # allocated on the producer thread's stream: keep the block out of its pool until
                # this stream is done with it
                self.tensor.record_stream(cur)
        return self.tensor

    def host(self) -> np.ndarray:
        if self._post is not None:
            self.post()
        if self._host_ev is not None:
            sync_event(self._host_ev, self.timeout_s, "sampled ids from the last stage")
            return self._host.numpy()
        t = self.wait()
        if t.is_cuda:
            return t.cpu().numpy()       # synchronises this stream; used off the hot path only
        return t.numpy()


def _elem_bytes(dtype) -> int:
    return torch.empty(0, dtype=dtype).element_size()


# per-hop traffic accounting (bytes per stage edge; bench JSON and /metrics): method ->
# (counter, bytes of one call from its arguments / result)
_COUNTED = {
    "send_hidden": ("hidden_tx", lambda a, r: a[0].numel() * a[0].element_size()),
    "recv_hidden": ("hidden_rx", lambda a, r: int(a[0]) * int(a[1]) * _elem_bytes(a[2])),
    "send_ids": ("ids_tx", lambda a, r: a[0].numel() * 4),
    "recv_ids": ("ids_rx", lambda a, r: int(a[0]) * 4),
    "send_meta": ("meta_tx", lambda a, r: 8 + 4 * len(a[0])),
    "recv_meta": ("meta_rx", lambda a, r: 8 + 4 * len(r)),
}
_hop_depth = threading.local()


def _counting(fn, key, size):
    @functools.wraps(fn)
    def wrapper(self, *a, **kw):
        depth = getattr(_hop_depth, "d", 0)
        _hop_depth.d = depth + 1
        try:
            r = fn(self, *a, **kw)
        finally:
            _hop_depth.d = depth
        if depth == 0:                    # outermost call only (a subclass may call super())
            h = self.__dict__.setdefault("_hop_bytes", {})
            h[key] = h.get(key, 0) + int(size(a, r))
        return r
    wrapper._counted = True
    return wrapper


class Transport:
    """Every subclass's send/recv methods are wrapped to count the bytes they move
    (:meth:`hop_stats`)."""
    stage: int
    num_stages: int

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        for name, (key, size) in _COUNTED.items():
            fn = cls.__dict__.get(name)
            if fn is not None and not getattr(fn, "_counted", False):
                setattr(cls, name, _counting(fn, key, size))

    def hop_stats(self) -> dict:
        """Bytes moved so far by this stage's transport: hidden / ids / meta, tx and rx."""
        return dict(self.__dict__.get("_hop_bytes", {}))

    def send_meta(self, arr: np.ndarray) -> None: ...
    def recv_meta(self) -> np.ndarray: ...
    def send_hidden(self, t: torch.Tensor) -> None: ...
    def recv_hidden(self, rows: int, hidden: int, dtype, device) -> torch.Tensor: ...
    def send_ids(self, ids: torch.Tensor) -> None: ...
    def recv_ids(self, n: int, device) -> PendingIds: ...


class DistTransport(Transport):
    """One pipeline = ranks ``ranks[0..pp-1]`` (global ranks), stage = index in that list."""

    kind = "torch"

    def __init__(self, ranks, stage: int, ctrl_group=None, data_group=None, ring_group=None, hop=None,
                 device=None, timeout_s: float = 600.0):
        """``data_group`` None = the default group (RCCL on GPU).  A gloo ``data_group`` with GPU
        stages means host-staged activations (D2H -> gloo -> H2D): the TCP fallback.
        ``ring_group``: the {first, last} group of this pipeline for the ids ring closure (None =
        the data group; fine wherever the activation and ids flows join different rank pairs).
        ``hop`` = (max rows, hidden, dtype, in-flight window): with GPU stages on the RCCL group the
        activations then use static send / receive rings of window + 1 slots (no clone, no
        allocation per hop; torch orders its RCCL stream after the compute stream at enqueue, so
        a receive into a slot follows that slot's previous consumers)."""
        self.ranks = list(ranks)
        self.timeout_s = float(timeout_s)
        self._tx = self._rx = None
        if hop is not None and device is not None and torch.device(device).type == "cuda" and data_group is None:
            rows, hidden, dtype, window = hop
            n = int(rows) * int(hidden)
            self._ring_n = window + 1
            self._tx = torch.empty(self._ring_n, n, dtype=dtype, device=device) if stage + 1 < len(ranks) else None
            self._rx = torch.empty(self._ring_n, n, dtype=dtype, device=device) if stage > 0 else None
            self._tx_work = [None] * self._ring_n
            self._tx_i = self._rx_i = 0
        self.ring = ring_group if ring_group is not None else data_group
        self._copy_stream = None
        self.stage = stage
        self.num_stages = len(self.ranks)
        self.ctrl = ctrl_group
        self.data = data_group
        self.prev = self.ranks[stage - 1] if stage > 0 else None
        self.next = self.ranks[stage + 1] if stage + 1 < self.num_stages else None
        self.first = self.ranks[0]
        self.last = self.ranks[-1]
        self._pending = []
        # GPU stages on the RCCL group: its p2p kernels spin on CUs like the native transport's, so
        # gemm_wide's split-K grids leave them room (ops/gemm.reserve_cus_for_comm)
        self._reserved_cus = (device is not None and torch.device(device).type == "cuda" and data_group is None
                              and dist.is_initialized() and dist.get_backend() == "nccl")
        if self._reserved_cus:
            from ..ops import gemm
            from .rccl_transport import comm_cus
            gemm.reserve_cus_for_comm(comm_cus())

    def close(self):
        if getattr(self, "_reserved_cus", False):
            from ..ops import gemm
            gemm.release_cus_for_comm()
            self._reserved_cus = False

    def _reap(self):
        # keep isend handles (and their buffers) alive until the transfer completed
        self._pending = [(w, t) for (w, t) in self._pending if not w.is_completed()]

    # ---- control (gloo, CPU tensors)
    def _send_arr(self, arr: np.ndarray, dst: int):
        arr = np.ascontiguousarray(arr, dtype=np.int32)
        hdr = torch.tensor([arr.shape[0]], dtype=torch.int64)
        body = torch.from_numpy(arr)
        self._pending.append((dist.isend(hdr, dst, group=self.ctrl), hdr))
        if arr.shape[0]:
            self._pending.append((dist.isend(body, dst, group=self.ctrl), body))
        self._reap()

    def _recv_arr(self, src: int) -> np.ndarray:
        hdr = torch.empty(1, dtype=torch.int64)
        dist.recv(hdr, src, group=self.ctrl)
        n = int(hdr.item())
        if n < 0:
            return np.array([STOP], dtype=np.int32)
        body = torch.empty(n, dtype=torch.int32)
        if n:
            dist.recv(body, src, group=self.ctrl)
        return body.numpy()

    def send_meta(self, arr):
        self._send_arr(arr, self.next)

    def recv_meta(self):
        return self._recv_arr(self.prev)

    def send_stop(self):
        if self.next is not None:
            hdr = torch.tensor([-1], dtype=torch.int64)
            dist.send(hdr, self.next, group=self.ctrl)

    # ---- ring closure: sampled ids, last stage -> stage 0
    def _ring_staged(self, device) -> bool:
        return torch.device(device).type == "cuda" and self.ring is not None \
            and dist.get_backend(self.ring) == "gloo"

    def send_ids(self, ids: torch.Tensor):
        ids = ids.to(torch.int32)
        if self._ring_staged(ids.device):
            ids = ids.to("cpu")                  # host-staged fallback
        else:
            ids = ids.clone()
        w = dist.isend(ids, self.first, group=self.ring)
        self._pending.append((w, ids))
        self._reap()

    def recv_ids(self, n: int, device) -> PendingIds:
        dev = torch.device(device)
        if self._ring_staged(dev):
            buf = torch.empty(n, dtype=torch.int32)
            w = dist.irecv(buf, self.last, group=self.ring)

            def fetch():
                w.wait()
                return buf.to(dev), None
            return PendingIds(fetch=fetch)
        buf = torch.empty(n, dtype=torch.int32, device=dev)
        w = dist.irecv(buf, self.last, group=self.ring)
        if dev.type == "cuda":
            if self._copy_stream is None:
                self._copy_stream = torch.cuda.Stream(dev)
            return PendingIds(buf, work=w, copy_stream=self._copy_stream, timeout_s=self.timeout_s)
        return PendingIds(buf, work=w, timeout_s=self.timeout_s)

    # ---- data plane (RCCL on GPU, gloo on CPU)
    def send_hidden(self, t: torch.Tensor):
        # copy: `t` may be a graph's static output that the next replay overwrites while the
        # send (on the comm stream) is still reading it
        if self._tx is not None and t.is_cuda and t.numel() <= self._tx.shape[1]:
            slot = self._tx_i % self._ring_n
            self._tx_i += 1
            if self._tx_work[slot] is not None:
                self._tx_work[slot].wait()       # stream-orders the overwrite after that send
            dst = self._tx[slot, : t.numel()]
            dst.copy_(t.reshape(-1))
            self._tx_work[slot] = dist.isend(dst, self.next, group=self.data)
            return
        if t.is_cuda and self.data is not None and dist.get_backend(self.data) == "gloo":
            t = t.to("cpu")                      # host-staged fallback (synchronous D2H)
        else:
            t = t.clone(memory_format=torch.contiguous_format)
        w = dist.isend(t, self.next, group=self.data)
        self._pending.append((w, t))
        self._reap()

    def recv_hidden(self, rows, hidden, dtype, device):
        if self._rx is not None and rows * hidden <= self._rx.shape[1] and dtype == self._rx.dtype:
            slot = self._rx_i % self._ring_n
            self._rx_i += 1
            buf = self._rx[slot, : rows * hidden]
            dist.irecv(buf, self.prev, group=self.data).wait()   # stream-ordered, no host block
            return buf.view(rows, hidden)
        staged = torch.device(device).type == "cuda" and self.data is not None \
            and dist.get_backend(self.data) == "gloo"
        buf = torch.empty(rows, hidden, dtype=dtype, device="cpu" if staged else device)
        dist.recv(buf, self.prev, group=self.data)
        return buf.to(device) if staged else buf

    def drain(self):
        for w, _ in self._pending:
            w.wait()
        self._pending = []
        if self._tx is not None:
            for w in self._tx_work:
                if w is not None:
                    w.wait()
            self._tx_work = [None] * self._ring_n

    def status(self) -> str:
        return ""


class LoopbackHub:
    """Shared queues for an in-process pipeline of ``num_stages`` stage threads."""

    def __init__(self, num_stages: int):
        self.num_stages = num_stages
        self.meta = [queue.Queue() for _ in range(num_stages)]     # into stage s
        self.hidden = [queue.Queue() for _ in range(num_stages)]
        self.ids = queue.Queue()

    def transport(self, stage: int) -> "LoopbackTransport":
        return LoopbackTransport(self, stage)


class LoopbackTransport(Transport):
    def __init__(self, hub: LoopbackHub, stage: int):
        self.hub, self.stage, self.num_stages = hub, stage, hub.num_stages

    def send_meta(self, arr):
        self.hub.meta[self.stage + 1].put(np.array(arr, copy=True))

    def recv_meta(self):
        return self.hub.meta[self.stage].get()

    def send_stop(self):
        if self.stage + 1 < self.num_stages:
            self.hub.meta[self.stage + 1].put(np.array([STOP], dtype=np.int32))

    def send_hidden(self, t):
        ev = None
        t = t.clone()
        if t.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        self.hub.hidden[self.stage + 1].put((t, ev))

    def recv_hidden(self, rows, hidden, dtype, device):
        t, ev = self.hub.hidden[self.stage].get()
        if ev is not None:
            cur = torch.cuda.current_stream()
            cur.wait_event(ev)
            # the producer thread drops its reference: without this the caching allocator may
            # hand the block to the producer's stream again while this stream still reads it
            t.record_stream(cur)
        assert t.shape == (rows, hidden), (t.shape, rows, hidden)
        return t

    def send_ids(self, ids):
        ids = ids.to(torch.int32).clone()
        ev = None
        if ids.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        self.hub.ids.put((ids, ev))

    def recv_ids(self, n, device) -> PendingIds:
        hub = self.hub

        def fetch():
            t, ev = hub.ids.get()
            if isinstance(t, BaseException):
                raise t
            assert t.shape[0] == n, (t.shape, n)
            return t, ev
        return PendingIds(fetch=fetch)

    def drain(self):
        pass
