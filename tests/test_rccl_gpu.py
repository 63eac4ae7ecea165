"""Native RCCL communicator (csrc/comm.hip) on a real GPU.

One GPU box: a 1-rank communicator exercises every entry point (RCCL runs a 1-rank
ring/all-reduce through its normal code path).  Two ranks sharing one device is attempted
too -- RCCL normally refuses duplicate devices in one communicator, in which case that case
is skipped (the 8-GPU path is exercised by the driver's multi-GPU runs).
"""
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def test_single_rank_comm_all_entry_points():
    from mercury_amd.parallel.rccl import RcclComm
    c = RcclComm()
    x = torch.randn(1001, device='cuda')
    ref = x.clone()
    c.allreduce(x, avg=True)
    c.ring_allreduce(x)
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    out = torch.empty(1001, device='cuda')
    c.all_gather(out, x)
    b = torch.arange(10, dtype=torch.int64, device='cuda')
    c.broadcast(b, 0)
    torch.cuda.synchronize()
    assert torch.equal(out, ref) and torch.equal(b.cpu(), torch.arange(10))
    c.close()


def _two_rank(rank, ws, q):
    from mercury_amd.parallel.rccl import RcclComm
    torch.cuda.set_device(0)
    try:
        c = RcclComm()
    except RuntimeError as e:          # duplicate device refused by RCCL
        q.put(('skip', str(e)))
        return
    x = torch.full((4099,), float(rank + 1), device='cuda')
    c.ring_allreduce(x)
    y = torch.full((77,), float(rank + 1), device='cuda')
    c.allreduce(y, avg=True)
    torch.cuda.synchronize()
    q.put(('ok', float(x.min()), float(x.max()), float(y[0])))


def test_two_ranks_one_device_ring():
    import torch.multiprocessing as mp
    from mercury_amd.parallel.dist import free_port
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()

    procs = [ctx.Process(target=_entry, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    import queue
    import time
    res, deadline = [], time.time() + 90
    while len(res) < 2 and time.time() < deadline:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break                      # a rank died: do not wait out the deadline
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert len(res) == 2, 'ranks exited %s' % [p.exitcode for p in procs]
    if any(r[0] == 'skip' for r in res):
        pytest.skip('RCCL refuses two ranks on one device: ' + res[0][1][:120])
    for r in res:
        assert r[1] == 3.0 and r[2] == 3.0 and r[3] == 1.5, r


def _entry(rank, ws, port, q):
    import os
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        _two_rank(rank, ws, q)
    finally:
        dist.destroy_process_group()
