"""The data-parallel gradient AVERAGE of the native engine, pinned numerically.

Reference: `pytorch_collab.py:236-249` (flatten -> all_reduce(SUM) -> / world_size ->
unflatten).  Replica-identity checks cannot see a missing or doubled 1/W, or a bucket reduced
over the wrong slice: every rank would still end up with the same (wrong) gradient.  Here each
rank trains on a different shard, the engine's ``grad_probe`` records every bucket as the
backward left it and the whole flat gradient the optimizer reads, and the test checks

    post  ==  (pre_rank0 + pre_rank1) / 2        (exactly: gloo SUM of two, then x 0.5)

over every bucket, which together must tile the flat buffer.  Paths:

* two ranks (gloo, both on cuda:0 -- the reference's own topology), ProcessGroup reduce, the
  graph-replayed step and the eager segmented step (``_finish_work``'s SUM -> mean);
* one rank over the engine's RCCL communicator with the one-rank AVG issued: the chained
  executable (event nodes) and the segmented replays (post == pre), the bf16 wire (post ==
  bf16(pre)) and the ternary wire (post in {0, +-max|pre|} with the sign of pre);
* the ternary codec's mean over two emulated ranks is unbiased over 64 Philox streams (the HIP
  pack / unpack kernels the RCCL path runs, messages concatenated as the all-gather lays them
  out), and the start-up all-reduce calibration picks the bucket plan.
"""
import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu


def _probe(eng):
    rec = {'pre': {}, 'post': None}

    def probe(stage, i, t):
        if stage == 'pre':
            rec['pre'][i] = t.detach().clone()
        else:
            rec['post'] = t.detach().clone()
    eng.grad_probe = probe
    return rec


def _check_tiling(eng):
    spans = sorted(eng.bucket_plan().values())
    assert spans[0][0] == 0 and spans[-1][1] == eng.lw.total, spans
    for (a, b), (c, d) in zip(spans, spans[1:]):
        assert b == c and a < b, spans


def _avg_worker(rank, ws, use_graphs):
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    torch.cuda.set_device(0)
    x, y = synthetic_arrays(2000, 10, seed=5)
    lo = rank * 1000                                # disjoint shards: different gradients
    torch.manual_seed(3)
    net = ResNet18(10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, world_size=ws, bucket_bytes=4 << 20, seed=11 + rank,
                       use_graphs=use_graphs)
    try:
        plan = eng.bucket_plan()
        assert len(plan) > 2
        _check_tiling(eng)
        eng.set_shard(x[lo:lo + 1000], y[lo:lo + 1000])
        eng.broadcast_from(0)
        eng.prime()
        eng.step()
        if use_graphs:
            eng.build_graphs()
        rec = _probe(eng)
        for _ in range(2):
            eng.step()
        torch.cuda.synchronize()
        assert len(rec['pre']) == len(plan)
        spans = {i: se for i, se in enumerate(sorted(plan.values(), reverse=True))}
        for i, pre in sorted(rec['pre'].items()):
            parts = [torch.zeros_like(pre) for _ in range(ws)]
            dist.all_gather(parts, pre)
            # the ranks really differ (else the average could not be told from the sum)
            assert not torch.equal(parts[0], parts[1]), i
            s, e = spans[i]
            ref = (parts[0] + parts[1]) * 0.5
            got = rec['post'][s:e]
            assert torch.equal(got, ref), (i, float((got - ref).abs().max()),
                                           float((got - 2 * ref).abs().max()))
    finally:
        eng.close()


@pytest.mark.parametrize('use_graphs', [True, False], ids=['graphs', 'eager'])
def test_two_rank_gradient_is_the_mean(use_graphs):
    from mercury_amd.parallel import spawn
    spawn(_avg_worker, 2, args=(use_graphs,), backend='gloo')


def _init_nccl_w1():
    from mercury_amd.parallel.dist import free_port
    if dist.is_initialized():
        dist.destroy_process_group()
    dist.init_process_group('nccl', init_method='tcp://127.0.0.1:%d' % free_port(), rank=0,
                            world_size=1, device_id=torch.device('cuda', 0))


def _w1_engine(x, y, **kw):
    from mercury_amd.config import EngineOptions
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    torch.manual_seed(7)
    net = ResNet18(10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, seed=3, force_buckets=True, comm='rccl', **kw)
    eng.set_shard(x, y)
    eng.prime()
    eng.step()
    eng.build_graphs()
    return eng


def test_rccl_paths_one_rank_wire_formats():
    from mercury_amd.config import EngineOptions
    from mercury_amd.data.datasets import synthetic_arrays
    x, y = synthetic_arrays(2000, 10, seed=5)
    _init_nccl_w1()
    engs = []
    try:
        cases = {
            'chained': dict(opts=EngineOptions(rccl_one_rank=True, comm_events=True)),
            'segmented': dict(opts=EngineOptions(rccl_one_rank=True, comm_events=False)),
            'bf16': dict(wire_bf16=True, opts=EngineOptions(rccl_one_rank=True)),
            'ternary': dict(grad_compress='ternary', opts=EngineOptions(rccl_one_rank=True)),
        }
        for name, kw in cases.items():
            eng = _w1_engine(x, y, bucket_bytes=4 << 20, **kw)
            engs.append(eng)
            assert bool(eng._train_exec) == (name != 'segmented'), name
            _check_tiling(eng)
            rec = _probe(eng)
            eng.step()
            torch.cuda.synchronize()
            spans = dict(enumerate(sorted(eng.bucket_plan().values(), reverse=True)))
            assert len(rec['pre']) == len(spans), name
            for i, pre in rec['pre'].items():
                s, e = spans[i]
                got = rec['post'][s:e]
                if name in ('chained', 'segmented'):
                    assert torch.equal(got, pre), (name, i)
                elif name == 'bf16':
                    assert torch.equal(got, pre.to(torch.bfloat16).float()), (name, i)
                else:
                    m = float(pre.abs().max())
                    nz = got != 0
                    assert bool(((got.abs() - m).abs()[nz] <= 1e-6 * m).all()), (name, i)
                    assert bool((torch.sign(got[nz]) == torch.sign(pre[nz])).all()), (name, i)
                    # the kept fraction is |g| / max|g| in expectation
                    frac = float(nz.float().mean())
                    want = float((pre.abs() / m).mean())
                    assert abs(frac - want) < 5 * (want / got.numel()) ** 0.5 + 1e-3, (i, frac,
                                                                                     want)
    finally:
        for e in engs:
            e.close()
        dist.destroy_process_group()


def test_ternary_codec_two_rank_mean_unbiased():
    """tern_pack on two emulated ranks (own Philox seeds), the two messages laid out as RCCL's
    all-gather delivers them, tern_unpack with scale 1/2: over 64 streams the decoded mean
    converges to (g0 + g1) / 2 -- no bias, and a dropped or doubled 1/W fails at once."""
    from mercury_amd import ops
    from mercury_amd.parallel.compress import tern_words
    L = ops.lib()
    n = 4099
    torch.manual_seed(0)
    g = [torch.randn(n, device='cuda'), torch.randn(n, device='cuda') * 0.3 + 0.1]
    ref = (g[0] + g[1]) * 0.5
    nw = tern_words(n)
    msgs = torch.zeros(2 * nw, dtype=torch.int32, device='cuda')
    ws = torch.zeros(1, dtype=torch.float32, device='cuda')
    out = torch.zeros(n, device='cuda')
    acc = torch.zeros(n, dtype=torch.float64, device='cuda')
    S = 64
    st = ops.stream_ptr()
    for k in range(S):
        for r in range(2):
            L.tern_pack(ops.ptr(g[r]), n, ops.ptr(ws), 1000 + 17 * r, k, ops.ptr(msgs[r * nw:]),
                        st, 0)
        L.tern_unpack(ops.ptr(msgs), 2, n, 0.5, ops.ptr(out), st)
        acc += out.double()
    torch.cuda.synchronize()
    mean = acc / S
    # per-element variance of the mean of two ternary codes: (m_r |g_r| - g_r^2) / 4 per rank
    var = sum(float(gr.abs().max()) * gr.abs() - gr * gr for gr in g).double() / 4 / S
    z = (mean - ref.double()) / var.clamp_min(1e-12).sqrt()
    # (small keep-probabilities make single z heavy-tailed: bound the bulk, not the extreme)
    assert float(z.abs().max()) < 10.0
    assert 0.8 < float((z * z).mean()) < 1.25, float((z * z).mean())
    assert abs(float(z.mean())) < 8.0 / n ** 0.5
    # the total over all elements is unbiased too (a 1/W slip moves it by ~100 sigma)
    tot = float((mean - ref.double()).sum()) / float(var.sum()) ** 0.5
    assert abs(tot) < 5.0


def test_bucket_plan_from_calibration():
    """Start-up calibration (EngineOptions.bucket_calib='on') on the one-rank RCCL
    communicator: alpha / beta are fitted from timed all-reduces, the bucket size and the last
    bucket come from them, the last bucket holds only the leading blocks, and training matches
    the uncalibrated forced-bucket engine."""
    from mercury_amd.config import EngineOptions
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.parallel.buckets import plan_from_calibration
    x, y = synthetic_arrays(2000, 10, seed=5)
    _init_nccl_w1()
    engs = []
    try:
        e = _w1_engine(x, y, opts=EngineOptions(bucket_calib='on', rccl_one_rank=True))
        base = _w1_engine(x, y, opts=EngineOptions(bucket_calib='off', rccl_one_rank=True))
        engs += [e, base]
        cal = e.comm_calib
        assert cal is not None and base.comm_calib is None
        assert cal['alpha_us'] > 0 and cal['beta_gbps'] > 0 and len(cal['ms']) == 3
        bb, lb = plan_from_calibration(cal)
        assert e.bucket_bytes == bb == cal['bucket_bytes'] and e.last_bucket_bytes == lb
        _check_tiling(e)
        spans = sorted(e.bucket_plan().values())
        starts = e._block_starts()
        # the last bucket (the lowest offsets) ends at a block boundary within its budget
        assert spans[0][1] in starts and spans[0][1] * 4 <= lb
        assert len(spans) >= 2
        for _ in range(3):
            e.step()
            base.step()
        torch.cuda.synchronize()
        d = float((e.opt.p - base.opt.p).abs().max())
        assert np.isfinite(d) and d < 5e-2, d
    finally:
        for en in engs:
            en.close()
        dist.destroy_process_group()
