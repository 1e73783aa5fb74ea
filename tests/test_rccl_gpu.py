"""Native RCCL p2p module (csrc/comm/rccl_p2p.cpp) on one GPU: a single-rank communicator
exchanging with itself exercises the build, the unique-id bootstrap, stream-ordered
ncclSend/ncclRecv and abort (multi-rank runs need one GPU per rank: RCCL refuses duplicates)."""
import pytest
import torch

from distributed_llms_amd import _ext

pytestmark = pytest.mark.gpu


def test_native_rccl_is_torchs_rccl(cuda):
    m = _ext.rccl()
    v = m.version()
    assert v >= 22000 and len(m.unique_id()) == 128


def test_native_rccl_self_sendrecv_on_side_stream(cuda):
    m = _ext.rccl()
    comm = m.RcclComm(1, 0, m.unique_id(), torch.cuda.current_device())
    assert comm.alive and comm.nranks == 1 and comm.rank == 0
    x = torch.randn(1024, 4096, device="cuda").to(torch.bfloat16)
    y = torch.empty_like(x)
    side = torch.cuda.Stream()
    ev = torch.cuda.Event()
    ev.record()
    side.wait_event(ev)
    comm.sendrecv(x.data_ptr(), x.numel() * 2, 0, y.data_ptr(), y.numel() * 2, 0, side.cuda_stream)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    comm.abort()
    assert not comm.alive
    with pytest.raises(RuntimeError):
        comm.send(x.data_ptr(), 16, 0, side.cuda_stream)
