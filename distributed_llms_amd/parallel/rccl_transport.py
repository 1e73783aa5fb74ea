"""Pipeline transport over the native RCCL p2p module (``csrc/comm/rccl_p2p.cpp``).

Control messages (batch metadata, markers) stay on DistTransport's gloo path.  Activations travel
through one two-rank RCCL communicator per pipeline EDGE (stage s -> s + 1, an xGMI peer link),
each stage driving its incoming and outgoing edge on two dedicated comm streams -- a stage's
receive of microbatch n + 1 never queues behind its send of microbatch n.  The sampled-ids ring
closure (last stage -> stage 0) is a third two-rank communicator with its own streams and rings,
so the whole data plane runs on communicators this module owns (and aborts: abort()).

No allocation and no clone per hop (static rings, ``window + 1`` slots, sized once from the
pipeline's largest hop):

  send_hidden : [compute] wait until the tx slot's previous send finished -> copy the stage output
                (a graph-static buffer the next replay overwrites) into the slot -> event
                [send]    wait event -> ncclSend(slot) -> "sent" event for the slot
  recv_hidden : [compute] "consumed" event for the previously received slot (everything the stage
                enqueued since includes its consumer)
                [recv]    wait until this slot was consumed -> ncclRecv(slot) -> "landed" event
                [compute] wait "landed" -> the stage reads the slot in place

so no host thread waits on the GPU, and slot reuse is ordered by events, not by the allocator.
Communicators are non-blocking with a deadline (``timeout_s``): a peer that never joins, or dies
while a connection is set up, makes this rank raise instead of hanging; the driver's host waits
on the ids ring are bounded the same way (comm.PendingIds).
"""
from __future__ import annotations

import collections

import torch
import torch.distributed as dist

from .. import _ext
from .comm import DistTransport


class _HostStream:
    """CPU stage (stand-in communicators only): every transfer is synchronous, so the streams and
    events of the GPU path become no-ops with the same interface."""
    cuda_stream = 0

    def wait_event(self, ev):
        pass

    def synchronize(self):
        pass


class _HostEvent:
    def record(self, stream=None):
        pass

    def query(self):
        return True

    def synchronize(self):
        pass


_COMM_STREAMS = {}


def shares_queue(spin_stream, others, wait_s: float = 0.05) -> list:
    """Indices of the streams in ``others`` that share ``spin_stream``'s hardware queue: a receive
    that is never matched (the device stand-in's kernel: one workgroup, no LDS, released through its
    host-mapped abort word, 2 s deadline) spins on ``spin_stream`` while one small kernel goes on
    each other stream; those not finished after ``wait_s`` sit behind the spinner.  A few ms."""
    import ctypes
    import time
    k = _ext.kernels()
    chunk, nslots = 4096, 2
    dev = spin_stream.device
    words = k.p2p_host_words(2)
    try:
        wv = (ctypes.c_int * 2).from_address(words)
        inbox = torch.zeros(k.p2p_inbox_bytes(chunk, nslots), dtype=torch.uint8, device=dev)
        dst = torch.empty(256, dtype=torch.uint8, device=dev)
        bufs = [torch.zeros(64, device=dev) for _ in others]
        torch.cuda.synchronize(dev)
        k.p2p_standin(0, 0, 0, 0, dst.data_ptr(), inbox.data_ptr(), dst.numel(), 0, chunk, nslots, 1, words, 2.0,
                      words + 4, 0, spin_stream.cuda_stream)
        evs = []
        for b, o in zip(bufs, others):
            with torch.cuda.stream(o):
                b.add_(1)
                e = torch.cuda.Event()
                e.record(o)
            evs.append(e)
        t_end = time.monotonic() + wait_s
        while time.monotonic() < t_end and not all(e.query() for e in evs):
            time.sleep(0.001)
        blocked = [i for i, e in enumerate(evs) if not e.query()]
        wv[0] = 1                                  # release the spinner
        spin_stream.synchronize()
        for e in evs:
            e.synchronize()
        return blocked
    finally:
        torch.cuda.synchronize(dev)
        k.p2p_host_words_free(words)


_HELD_STREAMS = []         # native streams made by isolated_pool_streams (probe candidates too): never freed


def _native_stream(dev):
    """A normal-priority stream outside torch's pool (torch's 32 pool streams are dealt out
    round-robin, so a probed pool stream could later be handed to another user -- a graph capture
    stream, a ``torch.cuda.Stream()`` -- whose work would then queue behind a spinning receive).
    Held for the life of the process; None without the native comm module."""
    try:
        h = _ext.rccl_native().plain_stream(dev.index or 0)
    except Exception:                    # noqa: BLE001 - older module / no RCCL: pool stream
        return None
    st = torch.cuda.ExternalStream(h, device=dev)
    _HELD_STREAMS.append(st)
    return st


def isolated_pool_streams(device, n: int, compute=None, tries: int = 12) -> list:
    """``n`` streams on hardware queues shared with neither ``compute`` (default: the current
    stream) nor each other, picked by probing (:func:`shares_queue`).  HIP deals a process's
    streams over GPU_MAX_HW_QUEUES queues in creation order, so which stream lands where depends
    on every stream created before -- a receive or a send spinning in the compute stream's queue
    would stall the stage (profiles/round5_comm_queues.md).  The candidates are native streams
    owned here (:func:`_native_stream`; torch pool streams only without the native module), so
    a chosen stream is never handed to anyone else.  Falls back to unprobed streams when no kernel
    module or not enough free queues are available."""
    dev = torch.device(device)
    compute = compute or torch.cuda.current_stream(dev)

    def make():
        return _native_stream(dev) or torch.cuda.Stream(device=dev)

    chosen = []
    try:
        _ext.kernels()
    except Exception:                    # noqa: BLE001 - no native kernels: unprobed streams
        return [make() for _ in range(n)]
    for _ in range(n):
        pick = None
        for _ in range(tries):
            s = make()
            if not shares_queue(s, [compute] + chosen):
                pick = s
                break
        chosen.append(pick if pick is not None else make())
    return chosen


def comm_stream(device, role: str = "comm"):
    """The stream of one communication role ("send", "recv", "ring", "copy").

    HIP deals a process's streams over GPU_MAX_HW_QUEUES (4) hardware queues, and a queue runs in
    order: a receive kernel spinning in it (a posted ncclRecv whose peer has not sent yet) or a
    stream-wait on an event holds up every later kernel of every stream sharing that queue.
    Measured on MI355X (scripts/hwq_probe.py, profiles/round5_comm_queues.md):
      * torch pool streams (default, ``knobs.comm_queue = "pool"``): a spinner blocks the pool
        streams dealt to its queue -- RcclTransport picks its role streams by probing
        (:func:`isolated_pool_streams`), this function hands out an unprobed one;
      * high-priority streams (``"priority"``: one native stream per role, created once, never
        destroyed) each get a queue of their own -- but a spinning high-priority kernel starves
        normal-priority work: pp2 kept 73 % of IPC, and pp4 stalled until the spinners' deadlines;
      * CU-masked streams all share ONE queue with the default stream (not offered)."""
    from .. import knobs
    dev = torch.device(device)
    if knobs.K.comm_queue != "priority":
        return torch.cuda.Stream(device=dev)
    key = (dev.index or 0, role)
    st = _COMM_STREAMS.get(key)
    if st is None:
        h = _ext.rccl_native().priority_stream(dev.index or 0)
        st = _COMM_STREAMS[key] = torch.cuda.ExternalStream(h, device=dev)
    return st


# CUs a stage's spinning comm kernels may hold at once (receive + send + ids ring, a few channel
# workgroups each): gemm_wide's split-K grids leave them free (ops/gemm.reserve_cus_for_comm);
# knobs.comm_reserved_cus overrides it
COMM_CUS = 16


def comm_cus() -> int:
    """knobs.comm_reserved_cus (default COMM_CUS; 0: no reservation)."""
    from .. import knobs
    return max(0, int(knobs.K.comm_reserved_cus))


class RcclTransport(DistTransport):
    kind = "rccl"

    def __init__(self, ranks, stage: int, ctrl_group, device, max_rows: int, hidden: int, dtype=torch.bfloat16,
                 ring_group=None, window: int = 2, timeout_s: float = 600.0, loopback: bool = False,
                 max_ids: int = 0):
        """``window``: the most microbatches in flight (the rings get window + 1 slots).
        ``loopback``: test mode on ONE rank -- a single one-rank communicator serves both edges
        (stage 0 sends to itself); each send is deferred and issued together with the matching
        receive as one grouped exchange, the only legal form of a self send."""
        super().__init__(ranks, stage, ctrl_group=ctrl_group, data_group=None, ring_group=ring_group,
                         timeout_s=timeout_s)
        dev = torch.device(device)
        from . import rccl_standin
        self.host = dev.type != "cuda"
        if self.host and not rccl_standin.enabled():
            raise ValueError("RcclTransport needs a GPU stage (CPU stages: the stand-in communicators only)")
        if window < 1:
            raise ValueError("in-flight window must be >= 1")
        self.device = dev
        self._reserved = False
        self.timeout_s = float(timeout_s)
        self.slots = window + 1
        self.slot_elems = int(max_rows) * int(hidden)
        self.dtype = dtype
        self.loopback = loopback
        self.comm_in = self.comm_out = self.ring_out = self.ring_in = None
        first, last = stage == 0, stage == len(self.ranks) - 1
        di = -1 if self.host else (dev.index or 0)
        if loopback:
            self.m = _ext.rccl()
            self.comm_out = self.comm_in = self.m.RcclComm(1, 0, self.m.unique_id(), di, self.timeout_s)
            self.ring_out = self.ring_in = self.comm_out
            self.next = self.prev = self.ranks[0]
        else:
            # one unique id per communicator, made by its sender.  Every rank of the ctrl group
            # takes part in the exchange (any dp x pp layout) UNCONDITIONALLY: a rank whose module
            # or unique id failed contributes its error instead, so every rank sees the same table
            # and raises before any communicator is built (the caller's fallback agreement then
            # runs on all ranks; a rank that skipped the exchange would hang the others in it)
            mine, err = {"edge": b"", "ring": b""}, ""
            try:
                self.m = _ext.rccl()
                mine = {"edge": self.m.unique_id() if self.next is not None else b"",
                        "ring": self.m.unique_id() if last and not first else b""}
            except Exception as e:          # noqa: BLE001 - reported through the exchange
                err = f"{type(e).__name__}: {e}"
            allv = [None] * dist.get_world_size(group=ctrl_group)
            dist.all_gather_object(allv, (dist.get_rank(), mine, err), group=ctrl_group)
            bad = [(r, e) for r, _, e in allv if e]
            if bad:
                raise RuntimeError(f"native RCCL unavailable on rank(s) {bad}")
            table = {r: m for r, m, _ in allv}
            # ascending edge order on every rank (in-edge first), the ring last: the chain of
            # inits cannot deadlock
            if self.prev is not None:
                self.comm_in = self.m.RcclComm(2, 1, table[self.prev]["edge"], di, self.timeout_s)
            if self.next is not None:
                self.comm_out = self.m.RcclComm(2, 0, mine["edge"], di, self.timeout_s)
            if last and not first:
                self.ring_out = self.m.RcclComm(2, 0, mine["ring"], di, self.timeout_s)
            elif first and not last:
                self.ring_in = self.m.RcclComm(2, 1, table[self.last]["ring"], di, self.timeout_s)
        # comm role streams on hardware queues of their own (probed; knobs.comm_queue)
        roles = [r for r, c in (("send", self.comm_out), ("recv", self.comm_in)) if c is not None]
        if (self.ring_out or self.ring_in) and (loopback or self.host or self.ring_out):
            roles.append("ring")
        if self.ring_in is not None and not self.host:
            roles.append("copy")                  # the sampled ids' copy-out (PendingIds), probed too
        picked = self._role_streams(roles)
        self._copy_stream = picked.get("copy")
        self.send_stream = picked.get("send")
        self.recv_stream = picked.get("recv")
        if loopback:
            self.recv_stream = self.send_stream
        self.tx = torch.empty(self.slots, self.slot_elems, dtype=dtype, device=dev) if self.comm_out else None
        self.rx = torch.empty(self.slots, self.slot_elems, dtype=dtype, device=dev) if self.comm_in else None
        self._sent = [None] * self.slots          # per tx slot: event after its ncclSend
        self._consumed = [None] * self.slots      # per rx slot: event after its consumer was enqueued
        self._tx_n = 0
        self._rx_n = 0
        self._last_rx = None
        self._deferred = []                       # loopback: sends waiting for their receive
        # sampled-ids ring closure: int32 slots of max_ids, deeper than the in-flight window
        self.max_ids = int(max_ids or max_rows)
        self.id_slots = 2 * window + 2
        # ring stream: the last stage's ids sends only (stage 0 posts each ids receive lazily on
        # its compute stream, in front of the consumer: PendingIds(post=...))
        self.ring_stream = picked.get("ring")
        self.ids_tx = torch.empty(self.id_slots, self.max_ids, dtype=torch.int32, device=dev) if self.ring_out else None
        self.ids_rx = torch.empty(self.id_slots, self.max_ids, dtype=torch.int32, device=dev) if self.ring_in else None
        self._ids_sent = [None] * self.id_slots
        self._ids_users = [None] * self.id_slots   # per rx slot: the PendingIds of its last use
        self._ids_tx_n = self._ids_rx_n = 0
        self._ids_deferred = []
        self._ids_unposted = collections.deque()   # PendingIds whose receive is not enqueued yet
        # last: every communicator is built (an init failure above leaves no reservation behind --
        # the job then falls back to torch.distributed, whose kernels this reservation is not for)
        if not self.host and not loopback:
            from ..ops import gemm
            gemm.reserve_cus_for_comm(comm_cus())
            self._reserved = True

    # streams / events of this stage's device (no-op shims on a CPU stage)
    def _stream(self, role):
        return _HostStream() if self.host else comm_stream(self.device, role)

    def _role_streams(self, roles) -> dict:
        from .. import knobs
        if self.host or knobs.K.comm_queue == "priority" or not roles:
            return {r: self._stream(r) for r in roles}
        return dict(zip(roles, isolated_pool_streams(self.device, len(roles))))

    def _event(self):
        return _HostEvent() if self.host else torch.cuda.Event()

    def _cur(self):
        return _HostStream() if self.host else torch.cuda.current_stream(self.device)

    @property
    def comm_ranks(self):
        """Ranks of this stage's RCCL edge communicators (reported by bench.py)."""
        return [c.nranks for c in self._comms()]

    def _check_hop(self, numel, dtype):
        if numel > self.slot_elems or dtype != self.dtype:
            raise ValueError(f"hop of {numel} x {dtype} exceeds the RCCL ring slot ({self.slot_elems} x {self.dtype})")

    def send_hidden(self, t: torch.Tensor):
        self._check_hop(t.numel(), t.dtype)
        n = self._tx_n
        self._tx_n += 1
        slot = n % self.slots
        cur = self._cur()
        if self._sent[slot] is not None:
            cur.wait_event(self._sent[slot])      # the slot's previous send has left
        dst = self.tx[slot, : t.numel()]
        dst.copy_(t.reshape(-1))
        nbytes = t.numel() * t.element_size()
        ready = self._event()
        ready.record(cur)
        if self.loopback:
            self._deferred.append((slot, nbytes, ready))
            return
        self.send_stream.wait_event(ready)
        self.comm_out.send(dst.data_ptr(), nbytes, 1, self.send_stream.cuda_stream)
        sent = self._event()
        sent.record(self.send_stream)
        self._sent[slot] = sent

    def recv_hidden(self, rows, hidden, dtype, device):
        self._check_hop(rows * hidden, dtype)
        cur = self._cur()
        if self._last_rx is not None:             # everything enqueued so far consumed that slot
            ev = self._event()
            ev.record(cur)
            self._consumed[self._last_rx] = ev
        n = self._rx_n
        self._rx_n += 1
        slot = n % self.slots
        rs = self.recv_stream
        if self._consumed[slot] is not None:
            rs.wait_event(self._consumed[slot])
        buf = self.rx[slot, : rows * hidden]
        nbytes = rows * hidden * buf.element_size()
        if self.loopback:
            tslot, tbytes, ready = self._deferred.pop(0)
            if tbytes != nbytes:
                raise RuntimeError(f"loopback hop size mismatch: sent {tbytes} B, receiving {nbytes} B")
            rs.wait_event(ready)
            self.comm_out.sendrecv(self.tx[tslot].data_ptr(), tbytes, 0, buf.data_ptr(), nbytes, 0, rs.cuda_stream)
            sent = self._event()
            sent.record(rs)
            self._sent[tslot] = sent
        else:
            self.comm_in.recv(buf.data_ptr(), nbytes, 0, rs.cuda_stream)
        landed = self._event()
        landed.record(rs)
        cur.wait_event(landed)
        self._last_rx = slot
        return buf.view(rows, hidden)

    # ---- ring closure: sampled ids, last stage -> stage 0, on the ring communicator
    def send_ids(self, ids: torch.Tensor):
        n_ids = ids.shape[0]
        if n_ids > self.max_ids:
            raise ValueError(f"{n_ids} sampled ids exceed the ring slot ({self.max_ids})")
        n = self._ids_tx_n
        self._ids_tx_n += 1
        slot = n % self.id_slots
        cur = self._cur()
        if self._ids_sent[slot] is not None:
            cur.wait_event(self._ids_sent[slot])
        dst = self.ids_tx[slot, :n_ids]
        dst.copy_(ids.reshape(-1))
        ready = self._event()
        ready.record(cur)
        if self.loopback:
            self._ids_deferred.append((slot, n_ids, ready))
            return
        self.ring_stream.wait_event(ready)
        self.ring_out.send(dst.data_ptr(), n_ids * 4, 1, self.ring_stream.cuda_stream)
        sent = self._event()
        sent.record(self.ring_stream)
        self._ids_sent[slot] = sent

    def recv_ids(self, n_ids: int, device) -> "PendingIds":
        from .comm import PendingIds
        if n_ids > self.max_ids:
            raise ValueError(f"{n_ids} sampled ids exceed the ring slot ({self.max_ids})")
        n = self._ids_rx_n
        self._ids_rx_n += 1
        slot = n % self.id_slots
        if not self.loopback and not self.host:
            # deferred: enqueued on the consumer's stream when first needed (wait / host), after
            # every earlier receive -- p2p receives match in issue order.  The slot's previous
            # users (lookahead gathers, its host copy) are on that same stream, so stream order
            # protects the slot
            buf = self.ids_rx[slot, :n_ids]
            p = PendingIds(buf, timeout_s=self.timeout_s)
            p._post = lambda p=p: self._post_ids_through(p)
            self._ids_unposted.append(p)
            self._ids_users[slot] = p
            return p
        cur = self._cur()
        rs = self.ring_stream
        # the slot's previous ids: consumed by device work enqueued before now (lookahead gathers)
        # and by their host copy
        free = self._event()
        free.record(cur)
        rs.wait_event(free)
        old = self._ids_users[slot]
        if old is not None and old._host_ev is not None:
            rs.wait_event(old._host_ev)
        buf = self.ids_rx[slot, :n_ids]
        if self.loopback:
            tslot, tn, ready = self._ids_deferred.pop(0)
            if tn != n_ids:
                raise RuntimeError(f"loopback ids mismatch: sent {tn}, receiving {n_ids}")
            rs.wait_event(ready)
            self.ring_out.sendrecv(self.ids_tx[tslot].data_ptr(), tn * 4, 0, buf.data_ptr(), n_ids * 4, 0,
                                   rs.cuda_stream)
            sent = self._event()
            sent.record(rs)
            self._ids_sent[tslot] = sent
        else:
            self.ring_in.recv(buf.data_ptr(), n_ids * 4, 0, rs.cuda_stream)
        landed = self._event()
        landed.record(rs)
        if self.host:
            p = PendingIds(buf, timeout_s=self.timeout_s)      # the stand-in recv already landed it
        else:
            if self._copy_stream is None:
                self._copy_stream = self._stream("copy")
            p = PendingIds(buf, ready=landed, copy_stream=self._copy_stream, timeout_s=self.timeout_s)
        self._ids_users[slot] = p
        return p

    def _post_ids_through(self, p):
        """Enqueue the deferred ids receives up to and including ``p`` on the current stream."""
        while self._ids_unposted:
            q = self._ids_unposted[0]
            if q is not p:
                q.post()                       # earlier receive first (its own host copy too)
                continue
            self._ids_unposted.popleft()
            cur = torch.cuda.current_stream(self.device)
            self.ring_in.recv(p.tensor.data_ptr(), p.tensor.numel() * 4, 0, cur.cuda_stream)
            return
        raise RuntimeError("ids receive posted twice or out of order")

    def _comms(self):
        return list({id(c): c for c in (self.comm_in, self.comm_out, self.ring_in, self.ring_out)
                     if c is not None}.values())

    def status(self) -> str:
        """"" when every communicator is healthy, else the first communicator error."""
        for c in self._comms():
            if c is not None:
                s = c.status()
                if s and s != "in_progress":
                    return s
        return ""

    def drain(self):
        while self._ids_unposted:              # keep the ring's receive sequence complete
            self._ids_unposted[0].post()
        super().drain()
        for s in (self.send_stream, self.recv_stream, self.ring_stream):
            if s is not None:
                s.synchronize()

    def abort(self):
        """ncclCommAbort on every communicator of this stage: kernels still waiting on a dead
        peer return, so the process can tear down (membership change)."""
        for c in self._comms():
            c.abort()

    def close(self):
        self.drain()
        if self._copy_stream is not None:
            self._copy_stream.synchronize()
        for c in self._comms():
            c.destroy()
        self.comm_in = self.comm_out = self.ring_in = self.ring_out = None
        if self._reserved:
            from ..ops import gemm
            gemm.release_cus_for_comm()
            self._reserved = False
        # the comm streams live for the process (comm_stream): torch's allocators may still hold
        # blocks whose pending events were recorded on them -- destroying the CU-masked streams of
        # an earlier version here crashed every stage process at exit
