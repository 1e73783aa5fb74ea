"""Pipeline transport over HIP IPC peer writes (``csrc/comm/ipc_p2p.cpp``).

Activations between adjacent stages travel without RCCL: every receiving stage exports a ring of
``SLOTS`` activation slots plus one flag word per slot, every sending stage exports one credit
word per slot, and the neighbours map each other's exports once at start-up (handles exchanged
over the gloo control group).  Message n of an edge uses slot ``n % SLOTS`` for the
``k = n // SLOTS``-th time:

  sender   (comm stream)    wait for the compute stream's copy of the output
                            -> wait credit[slot] >= k      (the receiver freed use k - 1)
                            -> copy into the peer's slot   (xGMI; same-device IPC on one GPU)
                            -> flag[slot] := k + 1         (hipStreamWriteValue32 on the peer)
  receiver (compute stream) wait flag[slot] >= k + 1       (hipStreamWaitValue32: the command
                                                            processor waits, no wave spins)
                            -> the stage consumes the slot in place
                            -> at the NEXT receive: credit[slot] := k + 1 on the sender,
                               stream-ordered behind this message's consumers

so a hop costs one copy and two stream memory operations, with no proxy thread or
communication kernel, and no host thread on either side waits for the GPU.  Sequence numbers
only grow, so the words never need resetting between rounds; ``SLOTS >= 2`` makes the credit
chain deadlock-free (the credit for message n comes with the receipt of message n - SLOTS + 1).

The sampled-ids ring closure and the control messages keep their DistTransport paths.  Unlike
RCCL, IPC works between two processes on the SAME device, so the multi-process pipeline runs
device to device on the 1-GPU test box (``DLLM_TRANSPORT=ipc``; tests/test_pipeline_gpu.py).
"""
from __future__ import annotations

import collections

import torch
import torch.distributed as dist

from .. import _ext
from .comm import DistTransport

SLOTS = 3


class IpcTransport(DistTransport):
    def __init__(self, ranks, stage: int, ctrl_group, device, max_rows: int, hidden: int, dtype=torch.bfloat16,
                 ring_group=None, slots: int = SLOTS):
        super().__init__(ranks, stage, ctrl_group=ctrl_group, data_group=None, ring_group=ring_group)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("IpcTransport needs a GPU stage")
        if slots < 2:
            raise ValueError("the credit chain needs at least two slots")
        self.m = _ext.rccl()
        if not self.m.can_wait_value(dev.index or 0):
            raise RuntimeError("device does not support hipStreamWaitValue32")
        self.device = dev
        self.slots = slots
        self.max_rows, self.hidden, self.dtype = int(max_rows), int(hidden), dtype
        self.slot_elems = self.max_rows * self.hidden
        self.slot_bytes = self.slot_elems * torch.empty(0, dtype=dtype).element_size()
        self.comm_stream = torch.cuda.Stream(device=dev)
        self._inflight = collections.deque()        # (done event, staged output kept alive)
        self._tx_n = 0
        self._rx_n = 0
        self._rx_held = None                        # (slot, use) of the message being consumed
        self._opened = []
        # exports: the receive ring + flags (stage > 0), the credits (stage < last)
        exports = {}
        if stage > 0:
            self.rx = torch.empty(slots, self.slot_elems, dtype=dtype, device=dev)
            self.rx_flag = torch.zeros(slots, dtype=torch.int32, device=dev)
            exports["rx"] = self.m.ipc_handle(self.rx.data_ptr())
            exports["flag"] = self.m.ipc_handle(self.rx_flag.data_ptr())
        if self.next is not None:
            self.credit = torch.zeros(slots, dtype=torch.int32, device=dev)
            exports["credit"] = self.m.ipc_handle(self.credit.data_ptr())
        torch.cuda.synchronize(dev)                 # zeroed words land before a peer can read them
        world = dist.get_world_size(group=ctrl_group)
        allv = [None] * world
        me = dist.get_rank()
        dist.all_gather_object(allv, (me, {k: (bytes(h), int(o)) for k, (h, o) in exports.items()}), group=ctrl_group)
        table = dict(allv)
        if self.next is not None:
            peer = table[self.next]
            self.peer_rx = self._open(peer["rx"])
            self.peer_flag = self._open(peer["flag"])
        if stage > 0:
            self.peer_credit = self._open(table[self.prev]["credit"])

    def _open(self, exp):
        handle, off = exp
        base, ptr = self.m.ipc_open(handle, off, self.device.index or 0)
        self._opened.append(base)
        return ptr

    def _retire(self):
        while self._inflight and self._inflight[0][0].query():
            self._inflight.popleft()

    # ---- data plane
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
        if use > 0:
            self.m.wait_value32(s, self.credit.data_ptr() + 4 * slot, use)
        self.m.copy_async(self.peer_rx + slot * self.slot_bytes, buf.data_ptr(),
                          rows * self.hidden * buf.element_size(), s)
        self.m.write_value32(s, self.peer_flag + 4 * slot, use + 1)
        buf.record_stream(cs)
        done = torch.cuda.Event()
        done.record(cs)
        self._inflight.append((done, buf))
        self._retire()

    def _release_held(self, stream):
        if self._rx_held is not None:
            slot, use = self._rx_held
            self.m.write_value32(stream, self.peer_credit + 4 * slot, use + 1)
            self._rx_held = None

    def recv_hidden(self, rows, hidden, dtype, device):
        if rows > self.max_rows or hidden != self.hidden or dtype != self.dtype:
            raise ValueError(f"hop of ({rows}, {hidden}) {dtype} does not fit the IPC slot")
        cur = torch.cuda.current_stream(self.device).cuda_stream
        # the previous message's consumers are queued on this stream by now: free its slot
        self._release_held(cur)
        n = self._rx_n
        self._rx_n += 1
        slot, use = n % self.slots, n // self.slots
        self.m.wait_value32(cur, self.rx_flag.data_ptr() + 4 * slot, use + 1)
        self._rx_held = (slot, use)
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

