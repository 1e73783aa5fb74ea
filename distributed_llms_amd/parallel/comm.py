"""Pipeline transports: the data plane between stages.

Three message kinds flow along a pipeline:
  meta    stage s -> s+1   packed int32 HostBatch (block tables, slots, ...)   CPU, control group
  hidden  stage s -> s+1   [T, H] bf16 activations                            device, data group
  tokens  last  -> stage 0 sampled ids (ring closure for the next decode step) CPU, control group

``DistTransport`` rides on torch.distributed: activations on the default group (backend
"nccl" = RCCL over xGMI on MI355X, gloo on CPU) as point-to-point isend/recv, whose
launches torch orders against the compute stream with events; control messages on a
separate gloo group so they never serialise behind GPU work.  ``LoopbackTransport`` is
the same interface over in-process queues, so N stage threads can share one GPU
(NCCL-family libraries refuse two ranks of one communicator on one device) -- this is
how the pipeline schedule is exercised on the single-GPU test box.
"""
from __future__ import annotations

import queue
import threading
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

STOP = -1


class Transport:
    stage: int
    num_stages: int

    def send_meta(self, arr: np.ndarray) -> None: ...
    def recv_meta(self) -> np.ndarray: ...
    def send_hidden(self, t: torch.Tensor) -> None: ...
    def recv_hidden(self, rows: int, hidden: int, dtype, device) -> torch.Tensor: ...
    def send_tokens(self, arr: np.ndarray) -> None: ...
    def recv_tokens(self) -> np.ndarray: ...


class DistTransport(Transport):
    """One pipeline = ranks ``ranks[0..pp-1]`` (global ranks), stage = index in that list."""

    def __init__(self, ranks, stage: int, ctrl_group=None, data_group=None):
        """``data_group`` None = the default group (RCCL on GPU).  A gloo ``data_group`` with GPU
        stages means host-staged activations (D2H -> gloo -> H2D): the TCP fallback."""
        self.ranks = list(ranks)
        self.stage = stage
        self.num_stages = len(self.ranks)
        self.ctrl = ctrl_group
        self.data = data_group
        self.prev = self.ranks[stage - 1] if stage > 0 else None
        self.next = self.ranks[stage + 1] if stage + 1 < self.num_stages else None
        self.first = self.ranks[0]
        self.last = self.ranks[-1]
        self._pending = []

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

    def send_tokens(self, arr):
        self._send_arr(arr, self.first)

    def recv_tokens(self):
        return self._recv_arr(self.last)

    # ---- data plane (RCCL on GPU, gloo on CPU)
    def send_hidden(self, t: torch.Tensor):
        # copy: `t` may be a graph's static output that the next replay overwrites while the
        # send (on the comm stream) is still reading it
        if t.is_cuda and self.data is not None and dist.get_backend(self.data) == "gloo":
            t = t.to("cpu")                      # host-staged fallback (synchronous D2H)
        else:
            t = t.clone(memory_format=torch.contiguous_format)
        w = dist.isend(t, self.next, group=self.data)
        self._pending.append((w, t))
        self._reap()

    def recv_hidden(self, rows, hidden, dtype, device):
        staged = torch.device(device).type == "cuda" and self.data is not None \
            and dist.get_backend(self.data) == "gloo"
        buf = torch.empty(rows, hidden, dtype=dtype, device="cpu" if staged else device)
        dist.recv(buf, self.prev, group=self.data)
        return buf.to(device) if staged else buf

    def drain(self):
        for w, _ in self._pending:
            w.wait()
        self._pending = []


class LoopbackHub:
    """Shared queues for an in-process pipeline of ``num_stages`` stage threads."""

    def __init__(self, num_stages: int):
        self.num_stages = num_stages
        self.meta = [queue.Queue() for _ in range(num_stages)]     # into stage s
        self.hidden = [queue.Queue() for _ in range(num_stages)]
        self.tokens = queue.Queue()

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

    def send_tokens(self, arr):
        self.hub.tokens.put(np.array(arr, copy=True))

    def recv_tokens(self):
        return self.hub.tokens.get()

    def drain(self):
        pass
