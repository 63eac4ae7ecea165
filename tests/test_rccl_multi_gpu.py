"""RCCL data parallelism across REAL GPUs (one rank per device): runs when the box has >= 2
GPUs (the 8-GPU driver node), skips on a one-GPU box.  Same checks as the gloo test of
test_native_dp_gpu.py, over the engine's own RCCL communicator and comm stream: bucketed AVG
all-reduce between graph replays, replicas bit-identical, score all-gather, global EMA; also
the direct-xGMI two-shot and the ternary wire."""
import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


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


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason='needs >= 2 GPUs (one rank each)')
@pytest.mark.parametrize('comm,compress', [('rccl', None), ('xgmi', None), ('rccl', 'ternary')])
def test_rccl_dp_real_gpus(comm, compress):
    from mercury_amd.parallel import spawn
    ws = min(torch.cuda.device_count(), 4)
    spawn(_worker, ws, args=(comm, compress), backend='nccl')
