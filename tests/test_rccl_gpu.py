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


def test_nonblocking_comm_self_exchange(cuda):
    """timeout_s > 0 builds a non-blocking communicator (init and enqueues polled to a deadline)."""
    m = _ext.rccl()
    comm = m.RcclComm(1, 0, m.unique_id(), torch.cuda.current_device(), 30.0)
    assert comm.status() == ""
    x = torch.arange(4096, device="cuda", dtype=torch.int32)
    y = torch.zeros_like(x)
    comm.sendrecv(x.data_ptr(), x.numel() * 4, 0, y.data_ptr(), y.numel() * 4, 0,
                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    comm.destroy()


def test_absent_peer_times_out_instead_of_hanging(cuda):
    """A two-rank communicator whose peer never joins: the rank raises within its deadline
    (a rank whose peer is dead must exit non-zero, not hang)."""
    import time
    m = _ext.rccl()
    t0 = time.monotonic()
    with pytest.raises(RuntimeError, match="did not respond|failed"):
        m.RcclComm(2, 0, m.unique_id(), torch.cuda.current_device(), 4.0)
    assert time.monotonic() - t0 < 60


def test_rccl_transport_static_rings_loopback(cuda):
    """The pipeline's native RCCL transport class through its own code path on one rank (a
    one-rank communicator serves every edge; each send is paired with its receive as one grouped
    exchange): static tx / rx rings wrapped several times, outputs overwritten right after the
    send (graph-static buffers), receives consumed later on the compute stream, and the
    sampled-ids ring closure with host copies."""
    from distributed_llms_amd.parallel.rccl_transport import RcclTransport
    dev = torch.device("cuda", torch.cuda.current_device())
    t = RcclTransport([0], 0, None, dev, max_rows=64, hidden=256, window=2, timeout_s=60, loopback=True,
                      max_ids=64)
    assert t.kind == "rccl" and t.comm_ranks == [1] and t.slots == 3
    out = torch.empty(64, 256, device=dev, dtype=torch.bfloat16)      # the "graph output" buffer
    sums, want, pend, ids_want = [], [], [], []
    g = torch.Generator(device="cuda").manual_seed(0)
    for n in range(11):
        rows = 1 + (n * 7) % 64
        x = torch.randn(rows, 256, device=dev, generator=g).to(torch.bfloat16)
        out[:rows].copy_(x)
        t.send_hidden(out[:rows])
        out.fill_(-1.0)                                  # the next replay overwrites the output
        y = t.recv_hidden(rows, 256, torch.bfloat16, dev)
        sums.append(y.float().sum(dim=1))                # consumed on the compute stream, in place
        want.append(x.float().sum(dim=1))
        ids = torch.randint(0, 1000, (rows,), device=dev, dtype=torch.int32, generator=g)
        t.send_ids(ids)
        pend.append(t.recv_ids(rows, dev))
        ids_want.append(ids.cpu())
        if len(pend) > 2:                                # the driver reads ids two steps later
            p = pend.pop(0)
            assert torch.equal(torch.from_numpy(p.host()), ids_want.pop(0))
    for p, w in zip(pend, ids_want):
        assert torch.equal(torch.from_numpy(p.host()), w)
    torch.cuda.synchronize()
    for a, b in zip(sums, want):
        torch.testing.assert_close(a, b, rtol=0, atol=0)
    assert t.status() == ""
    t.close()
