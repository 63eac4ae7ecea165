"""Direct-xGMI two-shot all-reduce (csrc/xgmi.hip, parallel/xgmi.py) on one GPU.

* emulated peers: W = 2..8 local buffers stand for the W ranks' IPC-mapped exchange buffers;
  every emulated rank's all-gather must equal the fp64 mean of all inputs (fp32 wire) or the
  sum of bf16-rounded inputs rounded once more (bf16 wire);
* two processes on the same GPU exchange real IPC handles and run the production
  ``XgmiAllReduce`` end to end: with host barriers (gloo) and with the device-side flag barriers
  (system-scope stores into the peer's IPC-mapped flag area), three all-reduces in a row
  alternating the two exchange slots, then a trailing barrier (odd count);
* the engine's ``comm='xgmi'`` path at world size 1 (forced buckets) trains like the default.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('W', [2, 3, 4, 5, 8])
@pytest.mark.parametrize('bf16', [False, True])
def test_emulated_two_shot(W, bf16):
    from mercury_amd.parallel.xgmi import emulated_allreduce
    for n in (4, 1000, 1 << 16, 4 * 12345):
        g = torch.Generator(device='cpu').manual_seed(n + W)
        xs = [torch.randn(n, generator=g).cuda() for _ in range(W)]
        outs = emulated_allreduce(xs, avg=True, wire_bf16=bf16)
        torch.cuda.synchronize()
        if bf16:
            ref = torch.stack([x.to(torch.bfloat16).float() for x in xs]).sum(0) / W
            for o in outs:
                torch.testing.assert_close(o, ref.to(torch.bfloat16).float(), rtol=1e-2,
                                           atol=1e-2)
        else:
            ref = torch.stack([x.double() for x in xs]).mean(0).float()
            for o in outs:
                torch.testing.assert_close(o, ref, rtol=1e-5, atol=1e-6)
        for o in outs[1:]:
            assert torch.equal(o, outs[0])          # every rank ends with identical values


def _ipc_rank(rank, ws, port, q, bf16, barrier):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        torch.cuda.set_device(0)
        from mercury_amd.parallel.xgmi import XgmiAllReduce
        try:
            x = XgmiAllReduce(1 << 14, 'cuda', wire_bf16=bf16, barrier=barrier, timeout_s=20.0)
        except RuntimeError as e:
            q.put(('skip', str(e)))
            return
        dist.barrier()
        out = []
        ts = []
        for k in range(3):              # slots 0, 1, 0: slot reuse after the second barrier
            t = torch.full((1 << 14,), float(rank + 1 + 10 * k), device='cuda')
            t[::7] = -2.0 * (rank + 1) - k
            x.allreduce(t, avg=True, slot=k % 2)
            ts.append(t)
        x.end_step(3)
        torch.cuda.synchronize()
        x.check()
        for t in ts:
            out.append((float(t[1]), float(t[0]), float(t[2])))
        q.put(('ok', out))
        dist.barrier()
        x.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('bf16', [False, True])
@pytest.mark.parametrize('barrier', ['host', 'device'])
def test_two_process_ipc_same_gpu(bf16, barrier):
    import queue
    import time
    import torch.multiprocessing as mp
    from mercury_amd.parallel.dist import free_port
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_ipc_rank, args=(r, 2, port, q, bf16, barrier))
             for r in range(2)]
    for p in procs:
        p.start()
    res, deadline = [], time.time() + 100
    while len(res) < 2 and time.time() < deadline:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert len(res) == 2, 'ranks exited %s' % [p.exitcode for p in procs]
    if any(r[0] == 'skip' for r in res):
        pytest.skip('IPC unavailable on this box: ' + [r for r in res if r[0] == 'skip'][0][1])
    for r in res:
        for k, v in enumerate(r[1]):
            # round k: mean of (1, 2) + 10 k and of (-2 - k, -4 - k)
            a, b = 1.5 + 10 * k, -3.0 - k
            assert v == (a, b, a), (k, v)


def test_engine_xgmi_world1_matches_default():
    import torch.distributed as dist
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    from mercury_amd.parallel.dist import free_port
    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % free_port(), rank=0,
                            world_size=1, device_id=torch.device('cuda', 0))
    try:
        x, y = synthetic_arrays(3000, 10, seed=5)
        engs = []
        for kw in (dict(), dict(force_buckets=True, comm='xgmi'),
                   dict(force_buckets=True, comm='xgmi', wire_bf16=True)):
            torch.manual_seed(7)
            e = NativeEngine(ResNet18(10).cuda(), 'cuda', 32, 10, bucket_bytes=4 << 20, seed=3,
                             **kw)
            e.set_shard(x, y)
            e.prime()
            e.step()
            e.build_graphs()
            engs.append(e)
        assert engs[1].xgmi is not None and len(engs[1].bucket_plan()) > 1
        for _ in range(5):
            for e in engs:
                e.step()
        torch.cuda.synchronize()
        for e in engs[1:]:
            d = float((e.opt.p - engs[0].opt.p).abs().max())
            assert torch.isfinite(e.opt.p).all() and d < 5e-2, d
    finally:
        dist.destroy_process_group()


def _timeout_rank(rank, ws, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(ws))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        torch.cuda.set_device(0)
        from mercury_amd.parallel.xgmi import XgmiAllReduce, XgmiTimeout
        try:
            x = XgmiAllReduce(1 << 12, 'cuda', barrier='device', timeout_s=0.5)
        except RuntimeError as e:
            q.put(('skip', str(e)))
            return
        dist.barrier()
        if rank == 0:
            # the peer never arrives: both device barriers of the all-reduce give up after 0.5 s
            t = torch.ones(1 << 12, device='cuda')
            x.allreduce(t, avg=True, slot=0)
            torch.cuda.synchronize()
            try:
                x.check()
                q.put(('no-raise', None))
            except XgmiTimeout as e:
                q.put(('timeout', str(e)))
        else:
            q.put(('idle', None))
        dist.barrier()
        try:
            x.close(sync_peers=False)
        except XgmiTimeout:
            pass
    finally:
        dist.destroy_process_group()


def test_device_barrier_timeout_is_reported():
    """A peer that never reaches the device flag barrier: the barrier gives up after timeout_s
    and ``check()`` (which the engine runs in read_meters) raises XgmiTimeout naming the peer."""
    import queue
    import time
    import torch.multiprocessing as mp
    from mercury_amd.parallel.dist import free_port
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_timeout_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, deadline = [], time.time() + 100
    while len(res) < 2 and time.time() < deadline:
        try:
            res.append(q.get(timeout=2))
        except queue.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    assert len(res) == 2, 'ranks exited %s' % [p.exitcode for p in procs]
    if any(r[0] == 'skip' for r in res):
        pytest.skip('IPC unavailable on this box')
    kinds = sorted(r[0] for r in res)
    assert kinds == ['idle', 'timeout'], res
    assert 'peers [1]' in [r for r in res if r[0] == 'timeout'][0][1]


def test_engine_read_meters_raises_on_xgmi_timeout():
    """The engine surfaces a device-barrier timeout at its next host sync (read_meters)."""
    import torch.distributed as dist
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    from mercury_amd.parallel.dist import free_port
    from mercury_amd.parallel.xgmi import XgmiTimeout
    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % free_port(), rank=0,
                            world_size=1, device_id=torch.device('cuda', 0))
    try:
        x, y = synthetic_arrays(1000, 10, seed=5)
        e = NativeEngine(ResNet18(10).cuda(), 'cuda', 32, 10, bucket_bytes=4 << 20, seed=3,
                         force_buckets=True, comm='xgmi')
        e.set_shard(x, y)
        e.prime()
        e.step()
        e.read_meters()                       # clean
        e.xgmi._err.fill_(1 << 3)             # as the barrier kernel records a late peer 3
        with pytest.raises(XgmiTimeout, match='peers \\[3\\]'):
            e.read_meters()
        e.xgmi._err.zero_()
        e.close()
        with pytest.raises(RuntimeError, match='closed'):
            e.step()
    finally:
        dist.destroy_process_group()
