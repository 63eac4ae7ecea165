"""RCCL data parallelism across REAL GPUs (one rank per device).

Collected for W in {2, 4, every device}: on the 8-GPU driver node that is W = 2, 4 and 8 (the
whole node, the size the scaling bench runs at); on a one-GPU box every case skips.  Same checks
as the gloo test of test_native_dp_gpu.py, over the engine's own RCCL communicator and comm
stream: bucketed AVG all-reduce (each bucket issued on the comm stream right after the train-graph
segment that finishes it, behind that segment's event node of the chained train executable),
replicas bit-identical,
score all-gather, global EMA; also the direct-xGMI two-shot (experimental) and the ternary wire.

``test_rccl_collectives_real_gpus`` drives every ``RcclComm`` entry point across the ranks --
including the explicit ring (`util.py:280-324` counterpart) at odd counts, counts below W and
buffers at misaligned (non-16-byte) offsets -- against a host-side reference."""
import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu

NDEV = torch.cuda.device_count() if torch.cuda.is_available() else 0


def _sizes():
    out = []
    for w in (2, 4, max(NDEV, 2)):
        if w not in out:
            out.append(w)
    return out


def _need(ws):
    if NDEV < ws:
        pytest.skip('needs %d GPUs (one rank each), box has %d' % (ws, NDEV))


def _worker(rank, ws, comm, compress):
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.data.partition import dirichlet_partition
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    x, y = synthetic_arrays(6000, 10, seed=5)
    np.random.seed(102)
    shard = dirichlet_partition(y, ws, 0.5, 10)[rank]
    torch.manual_seed(100 + rank)
    net = ResNet18(10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, world_size=ws, bucket_bytes=4 << 20, seed=rank,
                       exchange_scores=compress is None, global_ema=compress is None,
                       comm=comm, grad_compress=compress)
    assert eng.comm is not None and eng.comm.size == ws
    eng.set_shard(x[shard], y[shard])
    eng.broadcast_from(0)
    eng.prime()
    eng.step()
    eng.build_graphs()
    for _ in range(5):
        eng.step()
    torch.cuda.synchronize()
    p = eng.opt.p.clone()
    gathered = [torch.zeros_like(p) for _ in range(ws)]
    dist.all_gather(gathered, p)
    for r in range(1, ws):
        assert torch.equal(gathered[0], gathered[r]), float((gathered[0] - gathered[r]).abs().max())
    assert np.isfinite(eng.read_meters()['loss_sum'])
    if compress is None:
        g = eng.score_exchange.wait()
        torch.cuda.synchronize()
        assert torch.equal(g[rank], eng.score_mode.losses.reshape(-1))


@pytest.mark.parametrize('ws', _sizes())
@pytest.mark.parametrize('comm,compress', [('rccl', None), ('xgmi', None), ('rccl', 'ternary')])
def test_rccl_dp_real_gpus(ws, comm, compress):
    _need(ws)
    from mercury_amd.parallel import spawn
    spawn(_worker, ws, args=(comm, compress), backend='nccl')


def _collectives(rank, ws):
    from mercury_amd.parallel.rccl import RcclComm
    c = RcclComm.shared()
    assert c.size == ws and c.rank == rank
    # explicit ring: odd counts, counts below W, misaligned (4-byte-offset) views
    for n in (1, ws - 1, 7, 1001, 4099, 65537):
        if n < 1:
            continue
        for off in (0, 1, 3):
            base = torch.zeros(n + off + 4, device='cuda')
            t = base[off:off + n]
            g = torch.Generator().manual_seed(17 * n + off)
            vals = [torch.randint(-8, 8, (n,), generator=g).float() for _ in range(ws)]
            t.copy_(vals[rank].cuda())
            base[:off].fill_(123.0)
            base[off + n:].fill_(-77.0)
            c.ring_allreduce(t)
            torch.cuda.synchronize()
            ref = torch.stack(vals).sum(0)
            assert torch.equal(t.cpu(), ref), (n, off)
            # bytes outside the view untouched
            assert bool((base[:off] == 123.0).all()) and bool((base[off + n:] == -77.0).all())
    # ring AVG and the RCCL collectives
    x = torch.full((4099,), float(rank + 1), device='cuda')
    c.ring_allreduce(x, avg=True)
    y = torch.full((77,), float(rank + 1), device='cuda')
    c.allreduce(y, avg=True)
    z = torch.full((33,), float(rank), dtype=torch.bfloat16, device='cuda')
    c.allreduce(z, avg=False)
    out = torch.empty(5 * ws, dtype=torch.int32, device='cuda')
    c.all_gather(out, torch.full((5,), rank, dtype=torch.int32, device='cuda'))
    b = torch.full((9,), rank, dtype=torch.int64, device='cuda')
    c.broadcast(b, root=ws - 1)
    torch.cuda.synchronize()
    mean = (ws + 1) / 2.0
    assert torch.allclose(x, torch.full_like(x, mean)) and torch.allclose(y, torch.full_like(y, mean))
    assert float(z[0]) == ws * (ws - 1) / 2
    assert out.cpu().tolist() == [r for r in range(ws) for _ in range(5)]
    assert b.cpu().tolist() == [ws - 1] * 9


@pytest.mark.parametrize('ws', _sizes())
def test_rccl_collectives_real_gpus(ws):
    _need(ws)
    from mercury_amd.parallel import spawn
    spawn(_collectives, ws, backend='nccl')
