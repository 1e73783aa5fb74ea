"""Pipeline transport over the native RCCL p2p module (``csrc/comm/rccl_p2p.cpp``).

Control messages (batch metadata, tokens, markers) stay on the gloo control group exactly as in
:class:`DistTransport`; activations go through a per-pipeline RCCL communicator on a DEDICATED
comm stream:

  send_hidden : copy the stage output on the compute stream (graph outputs are static buffers the
                next replay overwrites) -> event -> comm stream waits -> ncclSend
  recv_hidden : ncclRecv into a fresh buffer on the comm stream -> event -> compute stream waits

so a stage's next microbatch is never queued behind a transfer, and no host thread blocks on the
GPU.  The communicator's unique id is created by each pipeline's stage 0 and distributed over the
control group (all_gather: every rank participates once, any dp x pp layout).

Opt-in with ``DLLM_TRANSPORT=rccl`` (default: torch.distributed's RCCL process group).
"""
from __future__ import annotations

import collections

import torch
import torch.distributed as dist

from .. import _ext
from .comm import DistTransport


class RcclTransport(DistTransport):
    def __init__(self, ranks, stage: int, ctrl_group, device):
        super().__init__(ranks, stage, ctrl_group=ctrl_group, data_group=None)
        dev = torch.device(device)
        if dev.type != "cuda":
            raise ValueError("RcclTransport needs a GPU stage")
        self.device = dev
        m = _ext.rccl()
        uid = m.unique_id() if stage == 0 else b""
        allv = [None] * dist.get_world_size(group=ctrl_group)
        dist.all_gather_object(allv, (self.ranks[0], uid), group=ctrl_group)
        mine = next(u for (r0, u) in allv if r0 == self.ranks[0] and u)
        self.comm = m.RcclComm(len(self.ranks), stage, mine, dev.index or 0)
        self.comm_stream = torch.cuda.Stream(device=dev)
        self._inflight = collections.deque()        # (done event, tensor kept alive)

    def _retire(self):
        while self._inflight and self._inflight[0][0].query():
            self._inflight.popleft()

    def send_hidden(self, t: torch.Tensor):
        cur = torch.cuda.current_stream(self.device)
        buf = t.clone(memory_format=torch.contiguous_format)
        ready = torch.cuda.Event()
        ready.record(cur)
        self.comm_stream.wait_event(ready)
        self.comm.send(buf.data_ptr(), buf.numel() * buf.element_size(), self.stage + 1,
                       self.comm_stream.cuda_stream)
        done = torch.cuda.Event()
        done.record(self.comm_stream)
        buf.record_stream(self.comm_stream)
        self._inflight.append((done, buf))
        self._retire()

    def recv_hidden(self, rows, hidden, dtype, device):
        cur = torch.cuda.current_stream(self.device)
        buf = torch.empty(rows, hidden, dtype=dtype, device=self.device)
        # the buffer comes from the compute stream's pool: order the comm stream after its
        # allocation point, and tell the allocator the comm stream uses it
        alloc = torch.cuda.Event()
        alloc.record(cur)
        self.comm_stream.wait_event(alloc)
        self.comm.recv(buf.data_ptr(), buf.numel() * buf.element_size(), self.stage - 1,
                       self.comm_stream.cuda_stream)
        buf.record_stream(self.comm_stream)
        got = torch.cuda.Event()
        got.record(self.comm_stream)
        cur.wait_event(got)
        return buf

    def drain(self):
        super().drain()
        self.comm_stream.synchronize()
        self._inflight.clear()

    def abort(self):
        self.comm.abort()
