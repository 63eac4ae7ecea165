"""Native engine data parallelism and Trainer API on a real GPU.

Two ranks share cuda:0 over gloo (the reference's own topology: every rank on
GPU 0, `pytorch_collab.py:253,269-275`) -- one GPU box cannot host an RCCL
communicator with two ranks on one device; the 8-GPU RCCL run is the driver's
scaling bench.  Checks: broadcast init, bucketed all-reduce inside the graph-
replayed step, replicas bit-identical after several steps.
"""
import os

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _dp_worker(rank, ws):
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.data.partition import dirichlet_partition
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    torch.cuda.set_device(0)
    x, y = synthetic_arrays(6000, 10, seed=5)
    np.random.seed(102)
    shard = dirichlet_partition(y, ws, 0.5, 10)[rank]
    torch.manual_seed(100 + rank)             # different init per rank
    net = ResNet18(10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, world_size=ws, bucket_bytes=4 << 20, seed=rank,
                       exchange_scores=True, global_ema=True)
    assert len(eng.bucket_plan()) > 1
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
    assert torch.equal(gathered[0], gathered[1]), float((gathered[0] - gathered[1]).abs().max())
    m = eng.read_meters()
    assert np.isfinite(m['loss_sum'])
    # cross-worker score exchange: row r of the gathered matrix is rank r's pool scores
    g = eng.score_exchange.wait()
    torch.cuda.synchronize()
    assert torch.equal(g[rank], eng.score_mode.losses.reshape(-1))
    # global EMA: one normaliser shared by every rank
    emas = [torch.zeros(2, device='cuda') for _ in range(ws)]
    dist.all_gather(emas, eng.ema.clone())
    assert torch.equal(emas[0], emas[1])
    share = eng.global_share()
    assert abs(float(share.sum()) - 1.0) < 1e-5


def test_native_dp_two_ranks_gloo_same_gpu():
    from mercury_amd.parallel import spawn
    spawn(_dp_worker, 2, backend='gloo')


def test_native_trainer_api_checkpoint(tmp_path):
    from mercury_amd.ckpt import load_checkpoint, save_checkpoint
    from mercury_amd.collab import make_trainer
    from mercury_amd.config import Config
    from mercury_amd.data import load_cifar10_noniid
    from mercury_amd.models import ResNet18
    from mercury_amd.engine.native import NativeTrainer
    np.random.seed(102)
    pres, train, test = load_cifar10_noniid(1, 0.5, data_dir='/nonexistent')
    cfg = Config(num_epochs=1, max_samples=40, print_every=20, eval_every=0, log_dir=str(tmp_path))
    torch.manual_seed(0)
    net = ResNet18(10).cuda()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    tr = make_trainer(cfg, net, opt, train, pres[0], test, 'cuda')
    assert isinstance(tr, NativeTrainer)
    tr.fit(1)
    assert tr.step > 30
    tl, ta, vl, va = tr.evaluate(max_batches=4)
    assert np.isfinite(tl.average) and 0 <= va.accuracy <= 1
    # weights/data/label/index/pool-mean API of update_samples
    w, d, lab, idx, pm = tr.update_samples()
    assert d.shape == (32, 3, 32, 32) and w.shape == (32,) and lab.shape == (32,)
    path = save_checkpoint(tr, os.path.join(tmp_path, 'ck.pt'))
    sd = torch.load(path, weights_only=True)
    # reference-compatible model state dict
    ref = ResNet18(10)
    ref.load_state_dict(sd['model'])
    assert set(sd['optimizer']['state'][0].keys()) >= {'exp_avg', 'exp_avg_sq'}
    # resume into a fresh trainer reproduces the parameters
    torch.manual_seed(1)
    net2 = ResNet18(10).cuda()
    tr2 = make_trainer(cfg, net2, torch.optim.Adam(net2.parameters(), lr=1e-3), train, pres[0],
                       test, 'cuda')
    load_checkpoint(tr2, path)
    assert torch.equal(tr2.engine.opt.p, tr.engine.opt.p)
    assert torch.equal(tr2.engine.opt.v, tr.engine.opt.v)
    # HBM importance table: scored samples carry their latest loss and scoring step
    tab = tr.engine.table
    scored = tab.group > 0
    # (a confidently classified sample can score exactly 0.0 in fp32)
    assert int(scored.sum()) > 0 and bool((tab.importance[scored] >= 0).all())
    assert float(tab.importance[scored].sum()) > 0
    assert torch.equal(tr2.engine.table.importance, tab.importance)


def _trainer_worker(rank, ws, tmp):
    """One rank of the two-rank NativeTrainer run: different init per rank, fit -> replicas
    identical -> per-rank checkpoint -> a fresh trainer (another init) resumes to the same
    parameters and optimizer state."""
    from mercury_amd.ckpt import load_checkpoint, save_checkpoint
    from mercury_amd.collab import make_trainer
    from mercury_amd.config import Config
    from mercury_amd.data import load_cifar10_noniid
    from mercury_amd.engine.native import NativeTrainer
    from mercury_amd.models import ResNet18
    torch.cuda.set_device(0)
    np.random.seed(102)
    pres, train, test = load_cifar10_noniid(ws, 0.5, data_dir='/nonexistent')
    cfg = Config(num_epochs=1, max_samples=60 * ws, print_every=0, eval_every=0, log_dir=tmp)
    torch.manual_seed(100 + rank)                          # different init per rank
    net = ResNet18(10).cuda()
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    tr = make_trainer(cfg, net, opt, train, pres[rank], test, 'cuda')
    assert isinstance(tr, NativeTrainer) and tr.world_size == ws
    tr.fit(1)                                              # average_model: broadcast from rank 0
    assert tr.step > 20
    torch.cuda.synchronize()
    p = tr.engine.opt.p.clone()
    gathered = [torch.zeros_like(p) for _ in range(ws)]
    dist.all_gather(gathered, p)
    assert torch.equal(gathered[0], gathered[1]), float((gathered[0] - gathered[1]).abs().max())
    path = save_checkpoint(tr, os.path.join(tmp, 'ckpt_rank%d.pt' % rank))
    torch.manual_seed(7 + rank)
    net2 = ResNet18(10).cuda()
    tr2 = make_trainer(cfg, net2, torch.optim.Adam(net2.parameters(), lr=1e-3), train,
                       pres[rank], test, 'cuda')
    load_checkpoint(tr2, path)
    assert torch.equal(tr2.engine.opt.p, p)
    assert torch.equal(tr2.engine.opt.m, tr.engine.opt.m)
    assert tr2.step == tr.step and tr2.epoch == tr.epoch
    tr.engine.close()
    tr2.engine.close()


def test_native_trainer_two_ranks_fit_checkpoint_resume(tmp_path):
    """The reference train-loop API end to end on two ranks (gloo, both on cuda:0, the
    reference's own topology): fit with different per-rank inits keeps the replicas
    bit-identical, and each rank resumes from its own checkpoint."""
    from mercury_amd.parallel import spawn
    spawn(_trainer_worker, 2, args=(str(tmp_path),), backend='gloo')


def _init_nccl_w1():
    from mercury_amd.parallel.dist import free_port
    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % free_port(), rank=0,
                            world_size=1, device_id=torch.device('cuda', 0))


def _engine(x, y, **kw):
    from mercury_amd.config import EngineOptions
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    torch.manual_seed(7)
    net = ResNet18(10).cuda()
    kw.setdefault('opts', EngineOptions(rccl_one_rank=True))   # RCCL runs even at W = 1
    eng = NativeEngine(net, 'cuda', 32, 10, bucket_bytes=4 << 20, seed=3, **kw)
    eng.set_shard(x, y)
    eng.prime()
    eng.step()
    eng.build_graphs()
    return eng


def test_native_rccl_buckets_world1():
    """The RCCL data-parallel path executed on one GPU: backend nccl at W = 1 with the bucket
    all-reduces forced on.  Checks: the native communicator's AVG all-reduces run on the comm
    stream behind their segments (device timing sees every bucket), ProcessGroupNCCL's async
    AVG path too, the stream-order race detector stays clean, the score all-gather works, and
    training matches the unbucketed engine (AVG over one rank is the identity)."""
    from mercury_amd.data.datasets import synthetic_arrays
    x, y = synthetic_arrays(3000, 10, seed=5)
    _init_nccl_w1()
    try:
        base = _engine(x, y)
        runs = {'rccl': _engine(x, y, force_buckets=True, comm='rccl', check_order=True,
                                exchange_scores=True),
                'pg': _engine(x, y, force_buckets=True, comm='pg', check_order=True),
                'bf16': _engine(x, y, force_buckets=True, comm='rccl', wire_bf16=True),
                'xgmi': _engine(x, y, force_buckets=True, comm='xgmi'),
                'tern': _engine(x, y, force_buckets=True, comm='rccl', grad_compress='ternary')}
        e = runs['rccl']
        assert e.comm is not None and e.comm.size == 1 and len(e.bucket_plan()) > 1
        # the score all-gather rides an RCCL communicator of its own: no ProcessGroup work, and
        # it does not queue in front of the gradient buckets
        assert e.score_exchange.comm is not None and e.score_exchange.comm is not e.comm
        for name in ('rccl', 'bf16', 'xgmi', 'tern'):
            assert runs[name]._train_exec, name          # one chained train executable
        assert not runs['pg']._train_exec
        for _ in range(6):
            base.step()
            for r in runs.values():
                r.step()
        # one timed step: every bucket's all-reduce has a device span on the comm stream
        e.timer.on = True
        e.step()
        e.timer.on = False
        ph = e.timer.collect()
        assert len(ph['comm_buckets']) == len(e.bucket_plan()), ph
        assert ph['comm'] > 0 and ph['step'] > 0 and 0.0 <= ph['overlap'] <= 1.0
        assert abs(ph['critical'] - ph['step']) <= 0.1 * ph['step'] + 0.05, ph
        base.step()
        for name in ('pg', 'bf16', 'xgmi', 'tern'):
            runs[name].step()
        torch.cuda.synchronize()
        for name in ('rccl', 'pg'):
            n, first = runs[name].order_violations()
            assert n == 0, (name, first)
        g = e.score_exchange.wait()
        torch.cuda.synchronize()
        assert torch.equal(g[0], e.score_mode.losses.reshape(-1))
        tern = runs.pop('tern')          # lossy wire: finite, not close
        assert torch.isfinite(tern.opt.p).all()
        for name, r in runs.items():
            # atomics make the steps non-bitwise-reproducible; Adam moves each weight by at
            # most a few lr per step (bias-corrected early steps), so 8 steps stay well below 5e-2
            d = float((r.opt.p - base.opt.p).abs().max())
            assert torch.isfinite(r.opt.p).all() and d < 5e-2, (name, d)
        # the identity itself, on the native communicator
        gg = torch.randn(1 << 20, device='cuda')
        ref = gg.clone()
        e.comm.allreduce(gg, avg=True)
        torch.cuda.synchronize()
        assert torch.equal(gg, ref)
        for r in list(runs.values()) + [tern, base]:
            r.close()
    finally:
        dist.destroy_process_group()


def test_capture_beside_outstanding_processgroup_work():
    """Regression for the round-4 driver abort (SIGABRT on a native thread while engines were
    being captured after a 'pg' engine had left ProcessGroupNCCL works behind).  The
    ProcessGroupNCCL watchdog thread polls its works' events; a global-mode capture forbids that
    poll process-wide and the watchdog aborts.  Engines capture thread-locally after quiescing,
    so captures with PG works still listed -- the pg engine's buckets plus a batch of large async
    all-reduces issued by the test itself -- must be harmless, repeatedly."""
    from mercury_amd.data.datasets import synthetic_arrays
    x, y = synthetic_arrays(3000, 10, seed=5)
    _init_nccl_w1()
    try:
        pg = _engine(x, y, force_buckets=True, comm='pg')
        others = []
        for k in range(3):
            pg.step()                                  # bucket works in the watchdog's list
            big = torch.randn(1 << 22, device='cuda')
            works = [dist.all_reduce(big, async_op=True) for _ in range(16)]
            others.append(_engine(x, y, force_buckets=True, comm='rccl'))
            for w in works:
                w.wait()
        for _ in range(3):
            pg.step()
            for o in others:
                o.step()
        torch.cuda.synchronize()
        for o in others + [pg]:
            assert torch.isfinite(o.opt.p).all() and np.isfinite(o.read_meters()['loss_sum'])
        for o in others + [pg]:
            o.close()
    finally:
        dist.destroy_process_group()


def test_native_rccl_buckets_comm_events():
    """EngineOptions.comm_events: ONE train graph (the segment graphs as child nodes) with an
    event-record node after each bucket's backward segment, the host-issued all-reduces on the
    comm stream waiting on those nodes.  The stream-order checker proves every all-reduce started after its segment ticked
    in the same replay (a wait on a stale record would run it early), and training matches the
    unbucketed engine."""
    from mercury_amd.config import EngineOptions
    from mercury_amd.data.datasets import synthetic_arrays
    x, y = synthetic_arrays(3000, 10, seed=5)
    _init_nccl_w1()
    try:
        base = _engine(x, y)
        runs = {'rccl': _engine(x, y, force_buckets=True, comm='rccl', check_order=True,
                                opts=EngineOptions(comm_events=True, rccl_one_rank=True)),
                'xgmi': _engine(x, y, force_buckets=True, comm='xgmi',
                                opts=EngineOptions(comm_events=True, rccl_one_rank=True))}
        for r in runs.values():
            assert r._train_exec and len(r.bucket_plan()) > 1
        for _ in range(8):
            base.step()
            for r in runs.values():
                r.step()
        torch.cuda.synchronize()
        n, first = runs['rccl'].order_violations()
        assert n == 0, first
        for name, r in runs.items():
            d = float((r.opt.p - base.opt.p).abs().max())
            assert torch.isfinite(r.opt.p).all() and d < 5e-2, (name, d)
    finally:
        dist.destroy_process_group()


def test_order_checker_detects_missing_wait():
    """The race detector itself: a tail that runs before the scoring stream ticked is
    reported (slot 0), a correctly ordered one is not."""
    from mercury_amd import ops
    o = torch.zeros(16, dtype=torch.int32, device='cuda')
    L = ops.lib()
    s = ops.stream_ptr()
    L.order_check(ops.ptr(o), -1, 0, 0, 0, 0, 0, 0, s)       # score tick
    L.order_check(ops.ptr(o), 0, 3, 1, 1, 0, 3, 3, s)        # tail: expects o[0] == o[3] + 1
    L.order_check(ops.ptr(o), 0, 3, 1, 1, 0, 3, 3, s)        # second tail without a score tick
    torch.cuda.synchronize()
    v = o.tolist()
    assert v[4] == 1 and v[8] == 0 and v[9] == 1 and v[10] == 2 and v[3] == 2, v


def test_ring_add_kernel_odd_counts_and_alignment():
    """comm.hip's ring add (dst += src) on odd lengths and on 4-byte-misaligned slices."""
    from mercury_amd import ops
    for n in (1, 3, 5, 1001, 4099, 65537):
        for off in (0, 1, 3):
            a = torch.randn(n + 8, device='cuda')
            b = torch.randn(n + 8, device='cuda')
            ref = a.clone()
            ref[off:off + n] += b[2:2 + n] if off else b[off:off + n]
            src = b[2:2 + n] if off else b[off:off + n]
            ops.lib().add_f32(ops.ptr(a[off:off + n]), ops.ptr(src), n, ops.stream_ptr())
            torch.cuda.synchronize()
            assert torch.equal(a, ref), (n, off)


def test_mobilenetv2_buckets_keep_deferred_dw_reduces():
    """MobileNetV2 under forced RCCL buckets (W = 1): the depthwise wgrad reduces stay deferred
    and batched -- flushed before the bucket all-reduce that carries them -- and training
    matches the unbucketed engine."""
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    x, y = synthetic_arrays(2000, 100, seed=9)
    _init_nccl_w1()
    try:
        engs = []
        for kw in (dict(), dict(force_buckets=True, comm='rccl', bucket_bytes=1 << 20)):
            torch.manual_seed(11)
            net = build_model('mobilenetv2', 100).cuda()
            e = NativeEngine(net, 'cuda', 32, 10, seed=4, **kw)
            e.set_shard(x, y)
            e.prime()
            e.step()
            e.build_graphs()
            engs.append(e)
        dp = engs[1]
        assert dp.dp and len(dp.bucket_plan()) > 2
        # every depthwise reduce is issued by a flush (none left pending after a step)
        assert dp.train_mode.dw_pending == []
        for _ in range(4):
            for e in engs:
                e.step()
        torch.cuda.synchronize()
        d = float((dp.opt.p - engs[0].opt.p).abs().max())
        assert torch.isfinite(dp.opt.p).all() and d < 5e-2, d
    finally:
        dist.destroy_process_group()
