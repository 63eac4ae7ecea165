"""Native engine vs the PyTorch module: forward, IS-weighted backward, scoring, steps."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _cos(a, b):
    a, b = a.flatten().double(), b.flatten().double()
    return float((a @ b) / (a.norm() * b.norm() + 1e-30))


def _engine(net, hw=32, **kw):
    from mercury_amd.engine.native import NativeEngine
    eng = NativeEngine(net, DEV, batch_size=32, pool_batches=10, use_graphs=False,
                       image_hw=(hw, hw), **kw)
    rng = np.random.RandomState(0)
    eng.set_shard(rng.randint(0, 256, (1000, hw, hw, 3), dtype=np.uint8), rng.randint(0, 10, 1000))
    return eng


@pytest.mark.parametrize('arch,hw', [('resnet18', 32), ('resnet50', 32), ('mobilenetv2', 32),
                                     ('resnet50_imagenet', 64), ('resnet50_imagenet', 224)])
def test_train_forward_backward_matches_torch(arch, hw):
    """Every supported family incl. the ImageNet stem (7x7/2 conv + 3x3/2 max-pool)."""
    from mercury_amd import ops
    from mercury_amd.models import build_model
    torch.manual_seed(0)
    ncls = 100 if arch == 'mobilenetv2' else 10
    net = build_model(arch, ncls).to(DEV)
    eng = _engine(net, hw)
    tm = eng.train_mode
    x = torch.randn(32, 3, hw, hw, device=DEV).to(torch.bfloat16).float()
    y = torch.randint(0, ncls, (32,), device=DEV)
    w = torch.rand(32, device=DEV) + 0.5
    tm.input.copy_(ops.to_nhwc(x))
    tm.label.copy_(y.int())
    eng.isw.copy_(w)
    tm.stats_arena.zero_()
    out = eng.forward(tm)
    eng.head(tm, out, 'train', isw=eng.isw, meters=eng.meters)
    last = len(eng.lw.blocks) - 1
    ops.head_bwd(tm.pooled, tm.dlogits, eng._pview(eng.lw.fc_w), eng._pview(eng.lw.fc_w, True),
                 eng._pview(eng.lw.fc_b, True), tm.buf[last, 'dout'], 32, tm.final_hw,
                 tm.final_C, eng.classes)
    for bi in range(last, -1, -1):
        eng.backward_block(tm, bi)
    torch.cuda.synchronize()
    # torch reference in train mode (batch-stat BN), same weights
    net.train()
    net.zero_grad()
    logits = net(x)
    loss = (F.cross_entropy(logits, y, reduction='none') / w).mean()
    loss.backward()
    got_loss = eng.meters[0].item() / 32
    assert abs(got_loss - loss.item()) < 0.05 * abs(loss.item()) + 0.02, (got_loss, loss.item())
    # what plain PyTorch reaches in bf16 on the same problem sets the tolerance:
    # deep layers' gradients pass through ~20 bf16 BN/conv backward stages
    import copy
    nb = copy.deepcopy(net).to(torch.bfloat16)
    nb.zero_grad()
    lb = (F.cross_entropy(nb(x.to(torch.bfloat16)).float(), y, reduction='none') / w).mean()
    lb.backward()
    pb = dict(nb.named_parameters())
    worst = 0.0
    for s in eng.lw.segs:
        g = eng._to_torch_layout(s, eng.opt.g)
        ref = s.param.grad
        if ref.norm() < 1e-8:
            continue
        gb = pb[s.name].grad.float()
        err = float((g - ref).norm())
        err_tb = float((gb - ref).norm())
        # no worse than PyTorch's own bf16 run (some grads, e.g. the stem BN bias, are
        # near-cancelling sums where even torch-bf16 keeps little of the fp32 direction)
        worst = max(worst, err / max(err_tb, 1e-12))
        assert err <= max(2.5 * err_tb, 0.05 * float(ref.norm())), (s.name, err, err_tb)
    print(arch, 'worst grad error relative to torch-bf16', worst)


@pytest.mark.parametrize('persist_bn', ['0', '1', 'row'])
def test_scoring_ghost_bn_matches_ten_separate_forwards(persist_bn, monkeypatch):
    """(persist_bn: the intra-block BN + ReLU applied inside the persistent halo convs -- the
    per-tap and the row-step kernels, or the row-step kernel only)"""
    from mercury_amd.models import ResNet18
    monkeypatch.setenv('MERCURY_ENGINE_OPTS', 'persist_bn=' + persist_bn)
    torch.manual_seed(1)
    net = ResNet18(10).to(DEV)
    eng = _engine(net)
    sm = eng.score_mode
    if persist_bn == '1':
        assert any(k[1] == 'hconv_bn' and p[2] == 0 for k, p in sm.plan.items())
    if persist_bn != '0':
        assert any(k[1] == 'hconv_bn' and p[2] < 0 for k, p in sm.plan.items())
    if persist_bn == 'row':
        assert not any(k[1] == 'hconv_bn' and p[2] >= 0 for k, p in sm.plan.items())
    sm.stats_arena.zero_()
    from mercury_amd import ops
    ops.pool_build(eng.shard, eng.shard_labels, eng.ctrl, sm.input, sm.label, sm.index, 320, 32,
                   eng.seed)
    x = eng.forward(sm)
    eng.head(sm, x, 'score')
    torch.cuda.synchronize()
    data = sm.input[..., :3].permute(0, 3, 1, 2).float()
    ref = []
    net.train()
    with torch.no_grad():
        for j in range(10):  # the reference's 10 separate train-mode forwards
            o = net(data[j * 32:(j + 1) * 32])
            ref.append(F.cross_entropy(o, sm.label[j * 32:(j + 1) * 32].long(), reduction='none'))
    ref = torch.cat(ref)
    assert _cos(sm.losses, ref) > 0.995
    # the bound is what plain PyTorch reaches in bf16 on the same ten forwards (a per-sample
    # bias would shift the sampling probabilities: bound the mean error AND the signed mean)
    import copy
    nb = copy.deepcopy(net).to(torch.bfloat16)
    refb = []
    with torch.no_grad():
        for j in range(10):
            o = nb(data[j * 32:(j + 1) * 32].to(torch.bfloat16)).float()
            refb.append(F.cross_entropy(o, sm.label[j * 32:(j + 1) * 32].long(),
                                        reduction='none'))
    refb = torch.cat(refb)
    err = (sm.losses - ref).abs().mean().item()
    err_tb = (refb - ref).abs().mean().item()
    bias = (sm.losses - ref).mean().item()
    bias_tb = (refb - ref).mean().item()
    print('ghost-BN scoring vs fp32: mean |err| %.5f (torch-bf16 %.5f), bias %.5f (torch-bf16 '
          '%.5f)' % (err, err_tb, bias, bias_tb))
    assert err <= max(2.5 * err_tb, 0.01), (err, err_tb)
    assert abs(bias) <= max(2.5 * abs(bias_tb), 0.01), (bias, bias_tb)


@pytest.mark.parametrize('graphs', [False, True])
def test_steps_reduce_loss_and_graph_matches_eager(graphs):
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    x, y = synthetic_arrays(4000, 10, seed=3)
    torch.manual_seed(0)
    net = ResNet18(10).to(DEV)
    eng = NativeEngine(net, DEV, 32, 10, lr=1e-3, use_graphs=graphs)
    eng.set_shard(x, y)
    eng.prime()
    eng.step()
    if graphs:
        eng.build_graphs()
    losses = []
    for i in range(60):
        eng.meters[:3].zero_()
        eng.step()
        m = eng.read_meters()
        losses.append(m['loss_sum'] / m['count'])
    assert all(math.isfinite(v) for v in losses)
    assert np.mean(losses[-10:]) < np.mean(losses[:10]), losses
    assert int(eng.ctrl[2].item()) == 61
    # BN running stats moved (train + 10 scoring updates per step)
    u = eng.units[0]
    assert int(u.bn.num_batches_tracked.item()) == 61 * 11
    eng.sync_to_module()
    net.eval()
    loss, acc, n = eng.evaluate_arrays(x[:1000], y[:1000])
    with torch.no_grad():
        from mercury_amd import ops
        xx = torch.as_tensor(x[:1000]).to(DEV).permute(0, 3, 1, 2).float() / 255
        mean = torch.tensor([0.49139968, 0.48215827, 0.44653124], device=DEV).view(1, 3, 1, 1)
        std = torch.tensor([0.24703233, 0.24348505, 0.26158768], device=DEV).view(1, 3, 1, 1)
        lo = net(((xx - mean) / std).to(torch.bfloat16).float())
        ref_loss = F.cross_entropy(lo, torch.as_tensor(y[:1000]).to(DEV)).item()
    assert n == 1000 and abs(loss - ref_loss) < 0.05 * ref_loss + 0.05, (loss, ref_loss)


def test_uniform_baseline_keeps_running_stats_sane():
    """Uniform sampling scores no pool: running stats update from the train batch only
    (a stale score-group table would drive running_var to zero and break eval)."""
    from mercury_amd.models import build_model
    torch.manual_seed(0)
    net = build_model('resnet18', 10).to(DEV)
    eng = _engine(net, importance=False)
    eng.scoring = False
    eng.prime()
    for _ in range(30):
        eng.step()
    torch.cuda.synchronize()
    rv = net.bn1.running_var
    assert float(rv.min()) > 1e-3, float(rv.min())
    assert int(net.bn1.num_batches_tracked) == 30


def test_vgg_speech_native_matches_torch():
    """Speech VGG on the native engine: float (spectrogram-like) shard converted once to NHWC
    bf16, conv+bias+BN+ReLU units with 2x2 max-pools, flatten -> fc1 -> fc2 head on the
    native HIP head kernels (csrc/head.hip mlp_head_*); gradients vs PyTorch within the bf16 tolerance (conv biases: exactly zero under
    train-mode BN, torch returns float noise -- not compared)."""
    import copy
    from mercury_amd import ops
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import VGG
    torch.manual_seed(0)
    H, W = 32, 64                                  # 5 pools -> 1 x 2 x 512 = 1024 features
    net = VGG('VGG11', 30, in_features=1024).to(DEV)
    eng = NativeEngine(net, DEV, 32, 10, use_graphs=False, image_hw=(H, W))
    rng = np.random.RandomState(0)
    eng.set_shard(rng.randn(200, 1, H, W).astype(np.float32), rng.randint(0, 30, 200))
    tm = eng.train_mode
    x = torch.randn(32, 1, H, W, device=DEV).to(torch.bfloat16).float()
    y = torch.randint(0, 30, (32,), device=DEV)
    w = torch.rand(32, device=DEV) + 0.5
    tm.input.copy_(ops.to_nhwc(x))
    tm.label.copy_(y.int())
    eng.isw.copy_(w)
    for fs, _ in eng.train_segments():
        for f in fs:
            f()
    torch.cuda.synchronize()
    net.train()
    net.zero_grad()
    loss = (F.cross_entropy(net(x), y, reduction='none') / w).mean()
    loss.backward()
    assert abs(eng.meters[0].item() / 32 - loss.item()) < 0.05 * abs(loss.item()) + 0.02
    nb = copy.deepcopy(net).to(torch.bfloat16)
    nb.zero_grad()
    (F.cross_entropy(nb(x.to(torch.bfloat16)).float(), y, reduction='none') / w).mean().backward()
    pb = dict(nb.named_parameters())
    conv_bias = {u.b_seg.name for b in eng.lw.blocks for u in b.units}
    for s in eng.lw.segs:
        g = eng._to_torch_layout(s, eng.opt.g)
        if s.name in conv_bias:
            assert float(g.abs().max()) == 0.0
            continue
        ref = s.param.grad
        if ref.norm() < 1e-8:
            continue
        err = float((g - ref).norm())
        err_tb = float((pb[s.name].grad.float() - ref).norm())
        assert err <= max(2.5 * err_tb, 0.05 * float(ref.norm())), (s.name, err, err_tb)
    # eval path on float inputs + a few graph-replayed IS steps
    l0, a0, n0 = eng.evaluate_arrays(rng.randn(64, 1, H, W).astype(np.float32),
                                     rng.randint(0, 30, 64), batch=32)
    assert n0 == 64 and np.isfinite(l0)
    eng2 = NativeEngine(net, DEV, 32, 10, use_graphs=True, image_hw=(H, W))
    eng2.set_shard(rng.randn(200, 1, H, W).astype(np.float32), rng.randint(0, 30, 200))
    eng2.prime()
    eng2.step()
    eng2.build_graphs()
    for _ in range(5):
        eng2.step()
    torch.cuda.synchronize()
    assert np.isfinite(eng2.read_meters()['loss_sum'])


def test_tiny_shard_smaller_than_batch_cycles():
    """A Dirichlet shard can be smaller than one batch at large world size: the pool cycles
    the shard (every sample index stays in range) instead of failing."""
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    torch.manual_seed(0)
    net = build_model('resnet18', 10).to(DEV)
    eng = NativeEngine(net, DEV, 32, 10, use_graphs=False)
    rng = np.random.RandomState(1)
    eng.set_shard(rng.randint(0, 256, (10, 32, 32, 3), dtype=np.uint8), rng.randint(0, 10, 10))
    eng.prime()
    for _ in range(3):
        eng.step()
    torch.cuda.synchronize()
    idx = eng.score_mode.index
    assert int(idx.min()) >= 0 and int(idx.max()) < 10
    assert sorted(set(idx[:10].tolist())) == list(range(10))    # one batch = a permutation, wrapped
    assert np.isfinite(eng.read_meters()['loss_sum'])


def test_step_tuner_keeps_engine_consistent():
    """In-situ plan tuner (ops/step_tune.py): every coordinate is a real plan of the engine,
    tuned plans land in its plan table, and the re-captured step still trains."""
    from mercury_amd.models import ResNet18
    from mercury_amd.ops import step_tune, tune
    torch.manual_seed(0)
    net = ResNet18(10).to(DEV)
    eng = _engine(net)
    eng.use_graphs = True
    eng.prime()
    eng.step()
    eng.build_graphs()
    coords = step_tune.coordinates(eng)
    kinds = {k for k, _, _ in coords}
    assert kinds == {'fwd', 'bwd'}
    res, base, final = step_tune.tune_step(eng, steps=2, chunks=1, budget_s=3.0,
                                           log=lambda s: None)
    assert res and base > 0 and final > 0
    for kind, key, users in coords:
        if key in res:
            m, name, _ = users[0]
            got = step_tune._get(kind, users)
            want = tuple(res[key]) if kind == 'fwd' else tuple(tuple(p) for p in res[key])
            assert got == want
    for _ in range(3):
        eng.step()
    assert math.isfinite(float(eng.read_meters()['loss_sum']))
    assert tune._key('fwd', coords[0][2][0][2]).startswith('fwd|')


@pytest.mark.parametrize('arch', ['resnet18', 'mobilenetv2'])
def test_head_applies_final_bn_in_pool(arch):
    """EngineOptions.head_bn: the scoring / eval head pools act(bn(y) [+ res]) straight from the
    last conv's output (no bn_apply pass).  Checked against a torch recompute from the SAME
    run's conv output, ghost statistics and residual (exact up to fp32 summation order), and
    against an engine that writes the block output first (losses to the bf16 rounding of that
    output and the run-to-run spread of atomically reduced statistics)."""
    from mercury_amd import ops
    from mercury_amd.config import EngineOptions
    from mercury_amd.models import build_model
    ncls = 100 if arch == 'mobilenetv2' else 10
    res = {}
    for on in (True, False):
        torch.manual_seed(2)
        net = build_model(arch, ncls).to(DEV)
        with torch.no_grad():
            for mod in net.modules():       # non-trivial running statistics for the eval pass
                if isinstance(mod, torch.nn.BatchNorm2d):
                    mod.running_mean.uniform_(-0.2, 0.2)
                    mod.running_var.uniform_(0.5, 2.0)
        eng = _engine(net, opts=EngineOptions(head_bn=on))
        sm = eng.score_mode
        sm.stats_arena.zero_()
        ops.pool_build(eng.shard, eng.shard_labels, eng.ctrl, sm.input, sm.label, sm.index, 320,
                       32, eng.seed)
        x = eng.forward(sm)
        assert (sm.head_bn is not None) == on
        eng.head(sm, x, 'score')
        torch.cuda.synchronize()
        if on:
            blk = eng.lw.blocks[-1]
            u = blk.units[-1]
            y = sm.buf[u.name, 'y'].float().view(10, 32, -1, u.K)
            st = sm.stats[u.name].view(10, 2, u.K)
            cnt = sm.spec[u.name].group_rows
            mean = st[:, 0] / cnt
            var = (st[:, 1] / cnt - mean * mean).clamp_min(0)
            sc = eng._gamma(u) / torch.sqrt(var + 1e-5)
            z = y * sc.view(10, 1, 1, u.K) + (eng._beta(u) - mean * sc).view(10, 1, 1, u.K)
            if sm.head_bn.get('res') is not None:
                z = z + sm.head_bn['res'].float().view(10, 32, -1, u.K)
            z = z.clamp(0, 6.0 if blk.final_act == 'relu6' else float('inf'))
            pref = z.mean(2).reshape(320, u.K)
            assert float((sm.pooled - pref).abs().max()) < 1e-4 * max(1.0, float(pref.abs().max()))
        rng = np.random.RandomState(3)
        ev = eng.evaluate_arrays(rng.randint(0, 256, (64, 32, 32, 3), dtype=np.uint8),
                                 rng.randint(0, ncls, 64), batch=64)
        res[on] = (sm.losses.clone(), ev)
        eng.close()
    (l1, e1), (l0, e0) = res[True], res[False]
    assert torch.isfinite(l1).all()
    assert float((l1 - l0).abs().mean()) < 2e-2 * max(1.0, float(l0.abs().mean()))
    assert abs(e1[0] - e0[0]) < 2e-2 * max(1.0, abs(e0[0])) and e1[2] == e0[2] == 64
