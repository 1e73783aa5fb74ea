"""Pipeline transport over HIP IPC peer writes (``csrc/comm/ipc_p2p.cpp``).

Activations between adjacent stages travel without RCCL: every receiving stage exports a ring of
activation slots plus one flag word per slot (hipIpcGetMemHandle), its upstream neighbour maps
them once at start-up (handles exchanged over the gloo control group).  Message n of an edge
uses slot ``n % slots`` for the ``k = n // slots``-th time:

  sender   (comm stream)    wait for the compute stream's staged copy of the output
                            -> copy into the peer's slot   (xGMI; same-device IPC on one GPU)
                            -> flag[slot] := k + 1         (hipStreamWriteValue32 on the peer)
  receiver (compute stream) wait flag[slot] >= k + 1       (hipStreamWaitValue32: the command
                                                            processor waits, no wave spins)
                            -> the stage consumes the slot in place

A hop is one copy and two stream memory operations -- no communication kernel, no proxy thread,
no host thread waiting on either side.  Sequence numbers only grow, so the words never need
resetting between rounds.

No credits flow back: the ring is deeper than the pipeline's in-flight window
(:func:`~distributed_llms_amd.parallel.pipeline.inflight_window`).  The driver issues
microbatch n only after microbatch n - window completed at stage 0 (its sampled ids came back),
i.e. after every stage's GPU finished it, so when a sender's copy of message n lands, the
previous user of its slot (message n - slots, slots > window) has long been consumed.  This is
deliberate: a credit wait would be a second command-processor wait on the SENDER's comm stream,
and HIP multiplexes a process's streams onto a few hardware queues (GPU_MAX_HW_QUEUES) -- a
blocked wait there can stall unrelated streams of that process behind it.  The only wait left is
the receiver's, on the stream that needs the data anyway.

The sampled-ids ring closure and the control messages keep their DistTransport paths.  Unlike
RCCL, IPC works between two processes on the SAME device, so the multi-process pipeline moves its
activations device to device on the 1-GPU test box (``DLLM_TRANSPORT=ipc``;
tests/test_pipeline_gpu.py).
"""
from __future__ import annotations

import collections

import torch
import torch.distributed as dist

from .. import _ext
from .comm import DistTransport


class IpcTransport(DistTransport):
    kind = "ipc"

    def __init__(self, ranks, stage: int, ctrl_group, device, max_rows: int, hidden: int, dtype=torch.bfloat16,
                 ring_group=None, window: int = 2):
        """``window``: the most microbatches in flight in the pipeline; the ring gets window + 1 slots."""
        super().__init__(ranks, stage, ctrl_group=ctrl_group, data_group=None, ring_group=ring_group)
        if window < 1:
            raise ValueError("in-flight window must be >= 1")
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("IpcTransport needs a GPU stage")
        self.m = _ext.rccl()
        if not self.m.can_wait_value(dev.index or 0):
            raise RuntimeError("device does not support hipStreamWaitValue32")
        self.device = dev
        self.slots = window + 1
        self.max_rows, self.hidden, self.dtype = int(max_rows), int(hidden), dtype
        self.slot_elems = self.max_rows * self.hidden
        self.slot_bytes = self.slot_elems * torch.empty(0, dtype=dtype).element_size()
        self.comm_stream = torch.cuda.Stream(device=dev)
        self._inflight = collections.deque()        # (done event, staged output kept alive)
        self._tx_n = 0
        self._rx_n = 0
        self._opened = []
        exports = {}
        if stage > 0:                               # receive ring + flags
            self.rx = torch.empty(self.slots, self.slot_elems, dtype=dtype, device=dev)
            self.rx_flag = torch.zeros(self.slots, dtype=torch.int32, device=dev)
            exports["rx"] = self.m.ipc_handle(self.rx.data_ptr())
            exports["flag"] = self.m.ipc_handle(self.rx_flag.data_ptr())
        torch.cuda.synchronize(dev)                 # zeroed flags land before a peer can see them
        allv = [None] * dist.get_world_size(group=ctrl_group)
        me = dist.get_rank()
        dist.all_gather_object(allv, (me, {k: (bytes(h), int(o)) for k, (h, o) in exports.items()}), group=ctrl_group)
        table = dict(allv)
        if self.next is not None:
            peer = table[self.next]
            self.peer_rx = self._open(peer["rx"])
            self.peer_flag = self._open(peer["flag"])

    def _open(self, exp):
        handle, off = exp
        base, ptr = self.m.ipc_open(handle, off, self.device.index or 0)
        self._opened.append(base)
        return ptr

    def _retire(self):
        while self._inflight and self._inflight[0][0].query():
            self._inflight.popleft()

    def send_hidden(self, t: torch.Tensor):
        rows = t.shape[0]
        if t.numel() > self.slot_elems or t.dtype != self.dtype:
            raise ValueError(f"hop of {tuple(t.shape)} {t.dtype} exceeds the IPC slot ({self.max_rows} x {self.hidden})")
        n = self._tx_n
        self._tx_n += 1
        slot, use = n % self.slots, n // self.slots
        cur = torch.cuda.current_stream(self.device)
        # stage outputs are graph-static buffers the next replay overwrites: stage a copy on the
        # compute stream, ship it from the comm stream
        buf = t.clone(memory_format=torch.contiguous_format)
        ready = torch.cuda.Event()
        ready.record(cur)
        cs = self.comm_stream
        cs.wait_event(ready)
        s = cs.cuda_stream
        self.m.copy_async(self.peer_rx + slot * self.slot_bytes, buf.data_ptr(),
                          buf.numel() * buf.element_size(), s)
        self.m.write_value32(s, self.peer_flag + 4 * slot, use + 1)
        buf.record_stream(cs)
        done = torch.cuda.Event()
        done.record(cs)
        self._inflight.append((done, buf))
        self._retire()

    def recv_hidden(self, rows, hidden, dtype, device):
        if rows * hidden > self.slot_elems or dtype != self.dtype:
            raise ValueError(f"hop of ({rows}, {hidden}) {dtype} does not fit the IPC slot")
        n = self._rx_n
        self._rx_n += 1
        slot, use = n % self.slots, n // self.slots
        cur = torch.cuda.current_stream(self.device).cuda_stream
        self.m.wait_value32(cur, self.rx_flag.data_ptr() + 4 * slot, use + 1)
        return self.rx[slot, : rows * hidden].view(rows, hidden)

    def drain(self):
        super().drain()
        self.comm_stream.synchronize()
        self._inflight.clear()

    def close(self):
        """Unmap the peers' exports (after the pipeline has drained)."""
        self.drain()
        torch.cuda.synchronize(self.device)
        for base in self._opened:
            self.m.ipc_close(base)
        self._opened = []
