"""HIP kernel numerics vs plain PyTorch fp32 references (SURVEY §4 layer 2).

Inputs are rounded to bf16 first so the reference sees exactly what the kernel
sees; tolerances then only cover bf16 output rounding / fp32 summation order.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = 'cuda'


def _ops():
    from mercury_amd import ops
    ops.lib()
    return ops


def bf(x):
    return x.to(torch.bfloat16).float()


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol + rtol * scale, 'max err %g (scale %g)' % (err, scale)


CONV_CASES = [
    # N, H, W, C, K, R, S, stride, pad
    (4, 32, 32, 3, 64, 3, 3, 1, 1),      # CIFAR stem (C padded to 8)
    (4, 32, 32, 64, 64, 3, 3, 1, 1),
    (4, 32, 32, 64, 128, 3, 3, 2, 1),
    (4, 32, 32, 64, 128, 1, 1, 2, 0),    # shortcut
    (8, 8, 8, 256, 512, 3, 3, 2, 1),     # small M -> split-K
    (32, 4, 4, 512, 512, 3, 3, 1, 1),    # layer4 at batch 32
    (2, 16, 16, 96, 24, 1, 1, 1, 0),     # MobileNet-style odd channels
    (2, 15, 15, 64, 128, 3, 3, 2, 1),    # odd input: uneven stride-2 dgrad parity classes
    (2, 15, 13, 64, 64, 1, 1, 2, 0),     # odd 1x1 stride-2 (three classes get no tap)
]


def _mk(case, seed=0):
    N, H, W, C, K, R, S, st, pd = case
    g = torch.Generator(device='cpu').manual_seed(seed)
    x = bf(torch.randn(N, C, H, W, generator=g)).to(DEV)
    w = bf(torch.randn(K, C, R, S, generator=g) / math.sqrt(C * R * S)).to(DEV)
    return x, w


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv_fwd_and_stats(case):
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    N, H, W, C, K, R, S, st, pd = case
    x, w = _mk(case)
    spec = ConvSpec(N, H, W, C, K, R, S, st, pd)
    xn = ops.to_nhwc(x)
    wk, _ = ops.pack_conv_weight(w)
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(2, K, device=DEV)
    plan = fwd_plan(spec)
    slab = torch.zeros(max(1, slab_bytes(spec.M, K, *plan) // 4), device=DEV)
    ops.conv_fwd(xn, wk, out, spec, stats=stats, slab=slab, plan=plan)
    ref = F.conv2d(x, w, stride=st, padding=pd)
    got = out.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2)
    close(got, ref)
    yb = bf(ref)
    close(stats[0], yb.sum((0, 2, 3)), rtol=1e-2, atol=0.5)
    close(stats[1], (yb * yb).sum((0, 2, 3)), rtol=1e-2, atol=0.5)


@pytest.mark.parametrize('bm_bn_split', [(128, 128, 1), (64, 64, 3), (128, 64, 2), (64, 128, 1),
                                         (256, 64, 1), (256, 128, 1), (256, 128, 3)])
def test_conv_fwd_all_tiles(bm_bn_split):
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, slab_bytes
    case = (4, 16, 16, 64, 128, 3, 3, 1, 1)
    x, w = _mk(case, 3)
    spec = ConvSpec(*case)
    out = torch.empty(spec.M, 128, dtype=torch.bfloat16, device=DEV)
    slab = torch.zeros(max(1, slab_bytes(spec.M, 128, *bm_bn_split) // 4), device=DEV)
    ops.conv_fwd(ops.to_nhwc(x), ops.pack_conv_weight(w)[0], out, spec, slab=slab,
                 plan=bm_bn_split)
    close(out.view(4, 16, 16, 128).permute(0, 3, 1, 2), F.conv2d(x, w, padding=1))


@pytest.mark.parametrize('case,gimgs', [((64, 8, 8, 64, 64, 3, 3, 1, 1), 32),
                                        ((12, 7, 9, 32, 64, 3, 3, 1, 1), 4),
                                        ((8, 11, 13, 64, 128, 3, 3, 1, 1), 2)])
def test_conv_ghost_group_stats(case, gimgs):
    """Per-group BN sums from the conv epilogue, incl. groups that are not a tile multiple
    (odd pixel counts: tiles straddle a group boundary)."""
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec
    N, K = case[0], case[4]
    G = N // gimgs
    x, w = _mk(case, 1)
    spec = ConvSpec(*case)
    spec.group_rows = gimgs * spec.P * spec.Q
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(G, 2, K, device=DEV)
    ops.conv_fwd(ops.to_nhwc(x), ops.pack_conv_weight(w)[0], out, spec, stats=stats)
    ref = bf(F.conv2d(x, w, padding=1))
    for gi in range(G):
        r = ref[gi * gimgs:(gi + 1) * gimgs]
        close(stats[gi, 0], r.sum((0, 2, 3)), rtol=1e-2, atol=0.5)
        close(stats[gi, 1], r.pow(2).sum((0, 2, 3)), rtol=1e-2, atol=0.5)


@pytest.mark.parametrize('case', [c for c in CONV_CASES if c[3] % 8 == 0])
def test_conv_dgrad(case):
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, slab_bytes
    N, H, W, C, K, R, S, st, pd = case
    x, w = _mk(case)
    spec = ConvSpec(N, H, W, C, K, R, S, st, pd)
    gy = bf(torch.randn(N, K, spec.P, spec.Q, device=DEV))
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, stride=st, padding=pd).backward(gy)
    _, wt = ops.pack_conv_weight(w)
    dx = torch.empty(N * H * W, spec.Cp, dtype=torch.bfloat16, device=DEV)
    plan = dgrad_plan(spec)
    slab = torch.zeros(max(1, slab_bytes(N * H * W, spec.Cp, *plan) // 4), device=DEV)
    ops.conv_dgrad(ops.to_nhwc(gy), wt, dx, spec, slab=slab, plan=plan)
    close(ops.from_nhwc(dx.view(N, H, W, spec.Cp), C), xr.grad)
    # accumulate mode adds onto existing contents
    dx2 = dx.clone()
    ops.conv_dgrad(ops.to_nhwc(gy), wt, dx2, spec, slab=slab, plan=plan, accumulate=True)
    close(ops.from_nhwc(dx2.view(N, H, W, spec.Cp), C), 2 * xr.grad, rtol=3e-2)


@pytest.mark.parametrize('case', [c for c in CONV_CASES if c[3] % 8 == 0])
@pytest.mark.parametrize('two', [False, True])
def test_conv_dgrad_fused_bn_backward_reduce(case, two):
    """dgrad epilogue reduces sum(dz), sum(dz*xhat) [, sum(dz*xhat2)] of its FINAL output
    (after accumulate), dz = dx * relu'(out) -- vs torch fp32 on the produced dx."""
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, slab_bytes
    N, H, W, C, K, R, S, st, pd = case
    x, w = _mk(case, 5)
    spec = ConvSpec(N, H, W, C, K, R, S, st, pd)
    Mx = N * H * W
    gy = ops.to_nhwc(bf(torch.randn(N, K, spec.P, spec.Q, device=DEV)))
    _, wt = ops.pack_conv_weight(w)
    plan = dgrad_plan(spec)
    slab = torch.zeros(max(1, slab_bytes(Mx, C, *plan) // 4), device=DEV)
    y = bf(torch.randn(Mx, C, device=DEV) * 2 + 0.5).to(torch.bfloat16)
    y2 = bf(torch.randn(Mx, C, device=DEV)).to(torch.bfloat16)
    out = bf(torch.relu(torch.randn(Mx, C, device=DEV))).to(torch.bfloat16)
    stats = torch.stack([y.float().sum(0), y.float().pow(2).sum(0)]).contiguous()
    stats2 = torch.stack([y2.float().sum(0), y2.float().pow(2).sum(0)]).contiguous()
    sums = torch.zeros(ops.sums_numel(C), device=DEV)
    prior = bf(torch.randn(Mx, C, device=DEV)).to(torch.bfloat16)
    dx = prior.clone()
    bw = dict(out=out, y=y, stats=stats, sums=sums, act='relu', eps=1e-5)
    if two:
        bw.update(y2=y2, stats2=stats2)
    ops.conv_dgrad(gy, wt, dx, spec, slab=slab, plan=plan, accumulate=True, bw=bw)
    d = dx.float()
    dz = d * (out.float() > 0)

    def xhat(t, s):
        mu = s[0] / Mx
        var = (s[1] / Mx - mu * mu).clamp_min(0)
        return (t.float() - mu) / torch.sqrt(var + 1e-5)
    ref0 = dz.sum(0)
    ref1 = (dz * xhat(y, stats)).sum(0)
    tot = ops.sums_total(sums, C)          # (the producers spread over SUMS_R replicas)
    close(tot[0], ref0, 1e-3, 1e-2)
    close(tot[1], ref1, 1e-3, 1e-2)
    if two:
        close(tot[2], (dz * xhat(y2, stats2)).sum(0), 1e-3, 1e-2)
    else:
        assert float(tot[2].abs().max()) == 0.0


@pytest.mark.parametrize('case', [c for c in CONV_CASES if c[3] % 8 == 0 and c[4] % 8 == 0])
def test_conv_bwd_pair_matches_separate_launches(case):
    """dgrad + wgrad in one launch == the two standalone kernels (bitwise for dx when K is not
    split, allclose for the atomically accumulated dw) and == torch."""
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, dgrad_plan, slab_bytes, wgrad_plan
    N, H, W, C, K, R, S, st, pd = case
    x, w = _mk(case, 3)
    spec = ConvSpec(N, H, W, C, K, R, S, st, pd)
    gy = bf(torch.randn(N, K, spec.P, spec.Q, device=DEV))
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=st, padding=pd).backward(gy)
    _, wt = ops.pack_conv_weight(w)
    dplan, wplan = dgrad_plan(spec), wgrad_plan(spec)
    Mx = N * H * W
    slab = torch.zeros(max(1, slab_bytes(Mx, spec.Cp, *dplan) // 4), device=DEV)
    xn, gyn = ops.to_nhwc(x), ops.to_nhwc(gy)
    dx = torch.empty(Mx, spec.Cp, dtype=torch.bfloat16, device=DEV)
    dw = torch.zeros(K * R * S * C, device=DEV)
    ops.conv_bwd(gyn, wt, dx, xn, dw, spec, dplan=dplan, wplan=wplan, slab=slab)
    dx2 = torch.empty_like(dx)
    dw2 = torch.zeros_like(dw)
    ops.conv_dgrad(gyn, wt, dx2, spec, slab=slab, plan=dplan)
    ops.conv_wgrad(gyn, xn, dw2, spec, plan=wplan)
    if dplan[2] == 1:
        assert torch.equal(dx, dx2)
    close(dx.float(), dx2.float(), 1e-2, 1e-2)
    close(dw, dw2, 1e-4, 1e-4)
    # the pair with the wgrad pixel splits reduced through a slab
    from mercury_amd.ops.conv import wgrad_slab_bytes
    wp2 = (64, 64, 4)
    wslab = torch.zeros(max(1, wgrad_slab_bytes(spec, wp2)) // 4 + 1, device=DEV)
    dw3 = torch.full_like(dw, 3.0)
    ops.conv_bwd(gyn, wt, dx2, xn, dw3, spec, dplan=dplan, wplan=wp2, slab=slab, wslab=wslab)
    close(dw3, dw2, 1e-4, 1e-4)
    close(ops.from_nhwc(dx.view(N, H, W, spec.Cp), C), xr.grad)
    close(dw.view(K, R, S, C).permute(0, 3, 1, 2), wr.grad, 2e-2, 2e-2)


@pytest.mark.parametrize('case', CONV_CASES)
def test_conv_wgrad(case):
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec
    N, H, W, C, K, R, S, st, pd = case
    if K % 8:
        pytest.skip('K % 8')
    x, w = _mk(case)
    spec = ConvSpec(N, H, W, C, K, R, S, st, pd)
    gy = bf(torch.randn(N, K, spec.P, spec.Q, device=DEV))
    wr = w.clone().requires_grad_(True)
    F.conv2d(x, wr, stride=st, padding=pd).backward(gy)
    dw = torch.zeros(K, R, S, C, device=DEV)
    ops.conv_wgrad(ops.to_nhwc(gy), ops.to_nhwc(x), dw, spec)
    close(dw.permute(0, 3, 1, 2), wr.grad, rtol=2e-2, atol=1e-2)
    from mercury_amd.ops.conv import wgrad_slab_bytes
    plans = [(64, 64, 1), (128, 128, 3), (64, 128, 2), (128, 64, 5)]
    wslab = torch.zeros(max(wgrad_slab_bytes(spec, p) for p in plans) // 4 + 1, device=DEV)
    for plan in plans:
        dw2 = torch.zeros_like(dw)
        ops.conv_wgrad(ops.to_nhwc(gy), ops.to_nhwc(x), dw2, spec, plan=plan)
        close(dw2, dw, rtol=1e-2, atol=1e-2)
        # split plans reduced through the slab (stores dw: a non-zero start is overwritten);
        # twice, so the tile counters the last arriver resets are exercised
        for _ in range(2):
            dw3 = torch.full_like(dw, 7.0)
            ops.conv_wgrad(ops.to_nhwc(gy), ops.to_nhwc(x), dw3, spec, plan=plan, slab=wslab)
            close(dw3, dw, rtol=1e-2, atol=1e-2)
    assert int(wslab[:1024].abs().sum()) == 0          # counters back at zero


def _bn_ref(y, gamma, beta, eps=1e-5):
    m = y.mean((0, 2, 3), keepdim=True)
    v = y.var((0, 2, 3), unbiased=False, keepdim=True)
    return (y - m) / torch.sqrt(v + eps) * gamma.view(1, -1, 1, 1) + beta.view(1, -1, 1, 1)


def test_bn_apply_and_bwd_with_bn_shortcut():
    ops = _ops()
    N, C, H, W = 8, 64, 8, 8
    M = N * H * W
    torch.manual_seed(0)
    y = bf(torch.randn(N, C, H, W, device=DEV) * 2 + 0.5)
    y2 = bf(torch.randn(N, C, H, W, device=DEV))
    g1, b1 = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    g2, b2 = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    yn, y2n = ops.to_nhwc(y).view(M, C), ops.to_nhwc(y2).view(M, C)
    st1 = torch.stack([y.sum((0, 2, 3)), (y * y).sum((0, 2, 3))])
    st2 = torch.stack([y2.sum((0, 2, 3)), (y2 * y2).sum((0, 2, 3))])
    out = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    ops.bn_apply(yn, st1, g1, b1, out, M, C, act='relu', res=y2n, res_bn=(st2, g2, b2))
    yr, y2r = y.clone().requires_grad_(True), y2.clone().requires_grad_(True)
    g1r, b1r, g2r, b2r = [t.clone().requires_grad_(True) for t in (g1, b1, g2, b2)]
    ref = F.relu(_bn_ref(yr, g1r, b1r) + _bn_ref(y2r, g2r, b2r))
    close(ops.from_nhwc(out.view(N, H, W, C)), ref)
    dout = bf(torch.randn_like(ref))
    ref.backward(dout)
    sums = torch.zeros(ops.sums_numel(C), device=DEV)
    dy = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    dy2 = torch.empty_like(dy)
    dz = torch.empty_like(dy)
    dg1, db1, dg2, db2 = [torch.zeros(C, device=DEV) for _ in range(4)]
    ops.bn_bwd(ops.to_nhwc(dout).view(M, C), out, yn, st1, g1, sums, dy, M, C, act='relu',
               y2=y2n, stats2=st2, gamma2=g2, dy2=dy2, dz=dz, dgamma=dg1, dbeta=db1,
               dgamma2=dg2, dbeta2=db2)
    close(ops.from_nhwc(dy.view(N, H, W, C)), yr.grad, rtol=3e-2, atol=3e-2)
    close(ops.from_nhwc(dy2.view(N, H, W, C)), y2r.grad, rtol=3e-2, atol=3e-2)
    close(dg1, g1r.grad, rtol=2e-2, atol=0.5)
    close(db1, b1r.grad, rtol=2e-2, atol=0.5)
    close(dg2, g2r.grad, rtol=2e-2, atol=0.5)
    close(db2, b2r.grad, rtol=2e-2, atol=0.5)


def test_bn_apply_ghost_groups_identity_residual_eval():
    ops = _ops()
    N, C, H, W = 64, 16, 4, 4
    M = N * H * W
    y = bf(torch.randn(N, C, H, W, device=DEV))
    r = bf(torch.randn(N, C, H, W, device=DEV))
    g, b = torch.rand(C, device=DEV) + 0.5, torch.randn(C, device=DEV)
    st = torch.zeros(2, 2, C, device=DEV)
    for gi in range(2):
        yy = y[gi * 32:(gi + 1) * 32]
        st[gi, 0], st[gi, 1] = yy.sum((0, 2, 3)), (yy * yy).sum((0, 2, 3))
    out = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    ops.bn_apply(ops.to_nhwc(y).view(M, C), st, g, b, out, M, C, group_rows=32 * 16, act='relu',
                 res=ops.to_nhwc(r).view(M, C))
    ref = torch.cat([F.relu(_bn_ref(y[i * 32:(i + 1) * 32], g, b) + r[i * 32:(i + 1) * 32])
                     for i in range(2)])
    close(ops.from_nhwc(out.view(N, H, W, C)), ref)
    rm, rv = torch.randn(C, device=DEV), torch.rand(C, device=DEV) + 0.5
    ops.bn_apply(ops.to_nhwc(y).view(M, C), None, g, b, out, M, C, act='relu6', running=(rm, rv))
    ref = F.relu6(F.batch_norm(y, rm, rv, g, b, False))
    close(ops.from_nhwc(out.view(N, H, W, C)), ref)


def test_bn_running_update_matches_torch():
    ops = _ops()
    C = 32
    bn = torch.nn.BatchNorm2d(C).to(DEV)
    xs = [bf(torch.randn(32, C, 4, 4, device=DEV) * 3 + 1) for _ in range(11)]
    for x in xs:
        bn(x)  # train mode: 11 momentum updates (1 train + 10 scoring)
    rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    nbt = torch.zeros(1, dtype=torch.int64, device=DEV)
    st = [torch.stack([x.sum((0, 2, 3)), (x * x).sum((0, 2, 3))]) for x in xs]
    st_train, st_score = st[0].contiguous(), torch.stack(st[1:]).contiguous()
    tab = ops.BnRunTable([(rm, rv, st_train, st_score, nbt, C, 1, 10, 512.0, 512.0)], DEV)
    tab.launch(0.1)
    close(rm, bn.running_mean, rtol=1e-4, atol=1e-4)
    close(rv, bn.running_var, rtol=1e-4, atol=1e-4)
    assert int(nbt.item()) == 11


def test_head_fwd_bwd_is_weighted():
    ops = _ops()
    B, HW, C, K = 32, 16, 512, 10
    act = bf(torch.rand(B, HW, C, device=DEV))
    w = torch.randn(K, C, device=DEV) * 0.05
    b = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (B,), device=DEV)
    isw = torch.rand(B, device=DEV) + 0.5
    pooled = torch.empty(B, C, device=DEV)
    dlog = torch.empty(B, K, device=DEV)
    losses = torch.empty(B, device=DEV)
    meters = torch.zeros(8, device=DEV)
    ops.head_fwd(act.to(torch.bfloat16), w, b, lab.int(), B, HW, C, K, 'train', pooled=pooled,
                 dlogits=dlog, losses=losses, isw=isw, meters=meters)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ar = act.clone().requires_grad_(True)
    logits = ar.mean(1) @ wr.t() + br
    l = F.cross_entropy(logits, lab, reduction='none')
    close(losses, l, rtol=1e-4, atol=1e-4)
    loss = (l / isw).mean()
    loss.backward()
    assert abs(meters[0].item() - loss.item() * B) < 1e-3 * B
    assert meters[2].item() == (logits.argmax(1) == lab).sum().item()
    dw, db = torch.empty_like(w), torch.empty_like(b)
    dact = torch.empty(B, HW, C, dtype=torch.bfloat16, device=DEV)
    ops.head_bwd(pooled, dlog, w, dw, db, dact, B, HW, C, K)
    close(dw, wr.grad, rtol=1e-3, atol=1e-5)
    close(db, br.grad, rtol=1e-3, atol=1e-5)
    close(dact, ar.grad, rtol=2e-2, atol=1e-5)


def test_head_gradnorm_score_matches_autograd():
    """score='gradnorm': per-sample classifier-layer gradient norm vs torch autograd."""
    ops = _ops()
    from mercury_amd.importance.pool import classifier_gradnorm
    B, HW, C, K = 16, 16, 512, 10
    act = bf(torch.rand(B, HW, C, device=DEV))
    w = torch.randn(K, C, device=DEV) * 0.05
    b = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (B,), device=DEV)
    losses = torch.empty(B, device=DEV)
    ops.head_fwd(act.to(torch.bfloat16), w, b, lab.int(), B, HW, C, K, 'score',
                 pooled=torch.empty(B, C, device=DEV), losses=losses, score='gradnorm')
    h = act.mean(1)
    ref = []
    for i in range(B):
        wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        F.cross_entropy((h[i:i + 1] @ wr.t() + br), lab[i:i + 1]).backward()
        ref.append(torch.sqrt(wr.grad.pow(2).sum() + br.grad.pow(2).sum()))
    ref = torch.stack(ref)
    close(losses, ref, rtol=1e-4, atol=1e-5)
    close(classifier_gradnorm(h @ w.t() + b, lab, h), ref, rtol=1e-4, atol=1e-5)


def test_is_sample_global_ema_over_gathered_scores():
    """Global-EMA mode: the replay runs over all ranks' cumulative pool means."""
    ops = _ops()
    from mercury_amd.importance.pool import global_cumulative_means
    from mercury_amd.utils import EMAverage
    P, B, W = 320, 32, 4
    g = torch.rand(W, P, device=DEV) * 3
    ema = torch.zeros(2, device=DEV)
    ctrl = torch.zeros(4, dtype=torch.int64, device=DEV)
    idx = torch.empty(B, dtype=torch.int32, device=DEV)
    w = torch.empty(B, device=DEV)
    meters = torch.zeros(8, device=DEV)
    ops.is_sample(g[1].contiguous(), ema, ctrl, idx, w, P, B, 32, seed=3, meters=meters,
                  gathered=g)
    ref = EMAverage()
    for j in range(10):
        ref.update(g[:, :32 * (j + 1)].mean().item())
    assert abs(ema[0].item() - ref.value) < 1e-5
    gm = global_cumulative_means(g, 32)
    assert abs(gm[-1].item() - g.mean().item()) < 1e-5
    assert abs(meters[3].item() - g.mean().item()) < 1e-5
    p = (g[1] + 0.5 * ema[0]) / (g[1] + 0.5 * ema[0]).sum()
    close(w, p[idx.long()] * P, rtol=1e-4, atol=1e-5)


def test_pool_build_epoch_permutation_and_normalisation():
    ops = _ops()
    from mercury_amd.data.transforms import CIFAR_MEAN, CIFAR_STD
    Ns, P, B = 100, 32, 16
    shard = torch.randint(0, 256, (Ns, 32, 32, 3), dtype=torch.uint8, device=DEV)
    labels = torch.arange(Ns, device=DEV) % 10
    ctrl = torch.zeros(4, dtype=torch.int64, device=DEV)
    pool = torch.empty(P, 32, 32, 8, dtype=torch.bfloat16, device=DEV)
    pl, pi = torch.empty(P, dtype=torch.int32, device=DEV), torch.empty(P, dtype=torch.int32, device=DEV)
    seen = []
    for pc in range(3):  # 6 batches of 16 = 96 = one epoch of 6 batches (drop_last of 100)
        ctrl[0] = pc
        ops.pool_build(shard, labels, ctrl, pool, pl, pi, P, B, seed=7, augment=False)
        seen += pi.tolist()
        assert torch.equal(pl.long(), labels[pi.long()])
    assert len(set(seen)) == 96  # no repeats inside an epoch
    # normalisation of the un-augmented view
    mean = torch.tensor(CIFAR_MEAN, device=DEV)
    std = torch.tensor(CIFAR_STD, device=DEV)
    ref = (shard[pi.long()].float() / 255 - mean) / std
    close(pool[..., :3].float(), ref, rtol=1e-2, atol=2e-2)
    assert pool[..., 3:].abs().max().item() == 0
    # augmented: crop+flip keeps values from the same image's value set or the pad value
    ops.pool_build(shard, labels, ctrl, pool, pl, pi, P, B, seed=7, augment=True)
    assert torch.isfinite(pool.float()).all()


@pytest.mark.parametrize('alias,P', [(True, 320), (False, 320), (True, 2048)])
def test_is_sample_ema_and_distribution(alias, P):
    """EMA replay exact; draws (parallel-built alias table or inverse CDF) match p by chi^2."""
    ops = _ops()
    from mercury_amd.utils import EMAverage
    B = 32
    torch.manual_seed(0)
    losses = torch.rand(P, device=DEV) ** 3 * 3      # skewed: many light, few heavy bins
    ema = torch.zeros(2, device=DEV)
    ctrl = torch.zeros(4, dtype=torch.int64, device=DEV)
    idx = torch.empty(B, dtype=torch.int32, device=DEV)
    w = torch.empty(B, device=DEV)
    ops.is_sample(losses, ema, ctrl, idx, w, P, B, 32, alpha=0.5, ema_alpha=0.9, seed=1,
                  alias=alias)
    ref = EMAverage()
    for j in range(P // 32):
        ref.update(losses[:32 * (j + 1)].mean().item())
    assert abs(ema[0].item() - ref.value) < 1e-5
    p = (losses + 0.5 * ema[0]) / (losses + 0.5 * ema[0]).sum()
    close(w, p[idx.long()] * P, rtol=1e-4, atol=1e-5)
    assert int(ctrl[0].item()) == 1
    counts = torch.zeros(P, device=DEV)
    n = 0
    for _ in range(600 * P // 320):
        ops.is_sample(losses, ema, ctrl, idx, w, P, B, 32, alpha=0.5, ema_alpha=0.9, seed=1,
                      alias=alias)
        counts.index_add_(0, idx.long(), torch.ones(B, device=DEV))
        n += B
    p = (losses + 0.5 * ema[0]) / (losses + 0.5 * ema[0]).sum()
    chi2 = ((counts / n - p) ** 2 / p).sum().item() * n
    assert chi2 < P + 6 * math.sqrt(2 * P), chi2


def test_gather_and_table_sampler():
    ops = _ops()
    P, B = 64, 8
    pool = torch.randn(P, 4, 4, 8, device=DEV).to(torch.bfloat16)
    pl = torch.arange(P, dtype=torch.int32, device=DEV)
    pi = pl * 3
    idx = torch.randint(0, P, (B,), dtype=torch.int32, device=DEV)
    batch = torch.empty(B, 4, 4, 8, dtype=torch.bfloat16, device=DEV)
    bl, bi = torch.empty(B, dtype=torch.int32, device=DEV), torch.empty(B, dtype=torch.int32, device=DEV)
    ops.gather(pool, pl, pi, idx, batch, bl, bi, B)
    assert torch.equal(batch, pool[idx.long()]) and torch.equal(bl, idx) and torch.equal(bi, idx * 3)


@pytest.mark.parametrize('N', [5000, 1_281_167])
def test_global_importance_table(N):
    """HBM table: contiguous write, index scatter with a device stamp, and the two-level
    inverse-CDF draw vs the exact distribution p ~ imp + mean(imp) over the group (chi^2)."""
    ops = _ops()
    torch.manual_seed(0)
    t = ops.ImportanceTable(N, DEV)
    lo, n = N // 3, 1000
    losses = torch.rand(n, device=DEV) * 4
    t.write(lo, losses, 3)
    assert torch.equal(t.importance[lo:lo + n], losses) and int(t.group[lo + 500]) == 3
    # scattered members far apart (other segments) stamped from a device scalar
    sidx = torch.randperm(N, device=DEV)[:200].to(torch.int32)
    sidx = sidx[(sidx < lo) | (sidx >= lo + n)]
    sl = torch.rand(sidx.numel(), device=DEV) * 2
    stamp = torch.full((1,), 3, dtype=torch.int64, device=DEV)
    t.scatter(sidx, sl, stamp=stamp)
    members = torch.cat([torch.arange(lo, lo + n, device=DEV), sidx.long()])
    imp = torch.cat([losses, sl])
    w = imp + imp.mean()
    p = (w / w.sum()).double()
    nd = 200_000
    out = t.sample(nd, 3, seed=5)
    mean, cnt, total = t.group_stats()
    assert cnt == members.numel() and abs(mean - imp.mean().item()) < 1e-4
    assert abs(total - w.sum().item()) / total < 1e-4
    lut = torch.full((N,), -1, dtype=torch.int64, device=DEV)
    lut[members] = torch.arange(members.numel(), device=DEV)
    pos = lut[out]
    assert int(pos.min()) >= 0, 'drew a non-member'
    counts = torch.bincount(pos, minlength=members.numel()).double()
    k = members.numel()
    chi2 = (((counts - nd * p) ** 2) / (nd * p)).sum().item()
    assert chi2 < k + 6 * math.sqrt(2 * k), chi2
    # the device draw counter advances -> a second batch differs
    out2 = t.sample(nd, 3, seed=5)
    assert not torch.equal(out, out2)
    # empty group -> -1
    assert int(t.sample(4, 99)[0]) == -1


def test_groupwise_sampler_gpu_lifecycle():
    from mercury_amd.importance.groupwise import Groupwise_Sampler

    class DS(object):
        def __len__(self):
            return 3000

    s = Groupwise_Sampler(DS(), device=DEV, seed=1, prefetch=64)
    s.update_importance(1, 1000, None, losses=torch.rand(1000) + 1)
    s.update_importance(1, 500, None, losses=torch.rand(500) + 1)   # same iteration -> same group
    draws = torch.as_tensor(list(iter(s)))
    assert draws.numel() == len(s) == 3000
    assert int(draws.min()) >= 0 and int(draws.max()) < 1500
    sd = s.state_dict()
    s2 = Groupwise_Sampler(DS(), device=DEV)
    s2.load_state_dict(sd)
    assert torch.equal(s2.importance, s.importance) and s2.group_index == 1


def test_fused_adam_matches_torch_and_writes_bf16_copies():
    ops = _ops()
    torch.manual_seed(0)
    conv = torch.randn(16, 8, 3, 3, device=DEV) * 0.1
    vec = torch.randn(10, device=DEV)
    k, c, r, s = conv.shape
    off2 = (conv.numel() + 3) // 4 * 4
    total = off2 + 12
    krsc = torch.zeros(k, r, s, c, dtype=torch.bfloat16, device=DEV)
    crsk = torch.zeros(c, r, s, k, dtype=torch.bfloat16, device=DEV)
    segs = [dict(off=0, numel=conv.numel(), kind=1, K=k, R=r, S=s, C=c, Cpad=c, w_krsc=krsc,
                 w_crsk=crsk),
            dict(off=off2, numel=10, kind=0)]
    opt = ops.FlatOptimizer(segs, total, DEV, 'adam', lr=1e-2, weight_decay=0.01)
    opt.p[:conv.numel()] = conv.permute(0, 2, 3, 1).reshape(-1)
    opt.p[off2:off2 + 10] = vec
    ref = [conv.clone().requires_grad_(True), vec.clone().requires_grad_(True)]
    topt = torch.optim.Adam(ref, lr=1e-2, weight_decay=0.01)
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    for t in range(5):
        g1, g2 = torch.randn_like(conv), torch.randn_like(vec)
        ref[0].grad, ref[1].grad = g1.clone(), g2.clone()
        topt.step()
        opt.g[:conv.numel()] = g1.permute(0, 2, 3, 1).reshape(-1)
        opt.g[off2:off2 + 10] = g2
        step += 1
        if t % 2:
            opt.step(step)
        else:   # split step (the engine's early optimizer): suffix first, then the prefix
            opt.step(step, start=off2)
            assert opt.g[:conv.numel()].abs().max().item() > 0   # prefix untouched so far
            opt.step(step, end=off2)
        assert opt.g.abs().max().item() == 0  # gradient consumed and zeroed
    close(opt.p[:conv.numel()].view(k, r, s, c).permute(0, 3, 1, 2), ref[0].detach(), 1e-5, 1e-6)
    close(opt.p[off2:off2 + 10], ref[1].detach(), 1e-5, 1e-6)
    close(krsc.float(), ref[0].detach().permute(0, 2, 3, 1), 1e-2, 1e-3)
    close(crsk.float(), ref[0].detach().permute(1, 2, 3, 0), 1e-2, 1e-3)
    with pytest.raises(ValueError):
        opt.step(step, start=3)          # not a segment start


@pytest.mark.parametrize('algo', ['adam', 'adamw', 'sgd'])
def test_fused_optimizer_tiles_match_torch(algo):
    """The one-launch step (64x64 update tiles writing both bf16 copies + elementwise rest):
    partial k / c tiles, a C % 4 != 0 conv (elementwise + transpose), a plain vector."""
    ops = _ops()
    torch.manual_seed(1)
    convs = [torch.randn(80, 96, 3, 3, device=DEV) * 0.1,     # partial k and c tiles
             torch.randn(128, 64, 1, 1, device=DEV) * 0.1,
             torch.randn(16, 6, 3, 3, device=DEV) * 0.1]      # C % 4 != 0
    vec = torch.randn(10, device=DEV)
    segs, off = [], 0
    copies = []
    for w in convs:
        k, c, r, s_ = w.shape
        krsc = torch.zeros(k, r, s_, c, dtype=torch.bfloat16, device=DEV)
        crsk = torch.zeros(c, r, s_, k, dtype=torch.bfloat16, device=DEV)
        segs.append(dict(off=off, numel=w.numel(), kind=1, K=k, R=r, S=s_, C=c, Cpad=c,
                         w_krsc=krsc, w_crsk=crsk))
        copies.append((krsc, crsk))
        off += (w.numel() + 3) // 4 * 4
    segs.append(dict(off=off, numel=10, kind=0))
    total = off + 12
    kw = dict(lr=1e-2, weight_decay=0.01)
    opt = ops.FlatOptimizer(segs, total, DEV, algo, momentum=0.9, **kw)
    assert opt.n_fjobs > 0 and opt.n_rest > 0
    for sg, w in zip(segs, convs):
        opt.p[sg['off']:sg['off'] + w.numel()] = w.permute(0, 2, 3, 1).reshape(-1)
    opt.p[off:off + 10] = vec
    ref = [w.clone().requires_grad_(True) for w in convs] + [vec.clone().requires_grad_(True)]
    topt = {'adam': lambda: torch.optim.Adam(ref, **kw),
            'adamw': lambda: torch.optim.AdamW(ref, **kw),
            'sgd': lambda: torch.optim.SGD(ref, momentum=0.9, **kw)}[algo]()
    step = torch.zeros(1, dtype=torch.int64, device=DEV)
    for t in range(4):
        gs = [torch.randn_like(r_) for r_ in ref]
        for r_, g_ in zip(ref, gs):
            r_.grad = g_.clone()
        topt.step()
        for sg, g_ in zip(segs[:-1], gs[:-1]):
            opt.g[sg['off']:sg['off'] + g_.numel()] = g_.permute(0, 2, 3, 1).reshape(-1)
        opt.g[off:off + 10] = gs[-1]
        step += 1
        opt.step(step)
        assert opt.g.abs().max().item() == 0
    for sg, w, r_, (krsc, crsk) in zip(segs, convs, ref, copies):
        k, c, r, s_ = w.shape
        got = opt.p[sg['off']:sg['off'] + w.numel()].view(k, r, s_, c).permute(0, 3, 1, 2)
        close(got, r_.detach(), 1e-5, 1e-6)
        close(krsc.float(), r_.detach().permute(0, 2, 3, 1), 1e-2, 1e-3)
        close(crsk.float(), r_.detach().permute(1, 2, 3, 0), 1e-2, 1e-3)
    close(opt.p[off:off + 10], ref[-1].detach(), 1e-5, 1e-6)


def test_quantize_pool_dwconv():
    ops = _ops()
    x = torch.randn(100000, device=DEV)
    q = ops.quantize(x, seed=3)
    m = x.abs().max()
    assert set(torch.unique(q.abs()).tolist()) <= {0.0, m.item()}
    acc = torch.zeros_like(x)
    for i in range(200):
        acc += ops.quantize(x, seed=3, counter=i)
    assert (acc / 200 - x).abs().mean().item() < 0.15
    # max pool 2x2 (VGG) and 3x3/s2/p1 (ImageNet stem), fwd + bwd
    for (k, st, pd) in [(2, 2, 0), (3, 2, 1)]:
        N, C, H, W = 2, 16, 12, 12
        xx = bf(torch.randn(N, C, H, W, device=DEV)).requires_grad_(True)
        ref = F.max_pool2d(xx, k, st, pd)
        P, Q = ref.shape[2:]
        y = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=DEV)
        am = torch.empty(N * P * Q * C, dtype=torch.uint8, device=DEV)
        ops.pool2d_fwd(ops.to_nhwc(xx.detach()), y, N, H, W, C, P, Q, k, st, pd, True, am)
        close(ops.from_nhwc(y), ref, 1e-3, 1e-3)
        gy = bf(torch.randn_like(ref))
        ref.backward(gy)
        dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
        ops.maxpool2d_bwd(ops.to_nhwc(gy), am, dx, N, H, W, C, P, Q, k, st, pd)
        close(ops.from_nhwc(dx), xx.grad, 1e-2, 1e-2)
    # depthwise 3x3, stride 1 and 2
    for st in (1, 2):
        N, C, H, W = 4, 24, 8, 8
        xx = bf(torch.randn(N, C, H, W, device=DEV)).requires_grad_(True)
        w = torch.randn(C, 1, 3, 3, device=DEV).requires_grad_(True)
        ref = F.conv2d(xx, bf(w), stride=st, padding=1, groups=C)
        P, Q = ref.shape[2:]
        y = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=DEV)
        stats = torch.zeros(2, C, device=DEV)
        wf = bf(w.detach()).reshape(C, 9).contiguous()
        ops.dwconv_fwd(ops.to_nhwc(xx.detach()), wf, y, N, H, W, C, P, Q, st, 1, stats=stats)
        close(ops.from_nhwc(y), ref)
        close(stats[0], bf(ref).sum((0, 2, 3)), 1e-2, 0.5)
        gy = bf(torch.randn_like(ref))
        ref.backward(gy)
        dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
        ops.dwconv_dgrad(ops.to_nhwc(gy), wf, dx, N, H, W, C, P, Q, st, 1)
        close(ops.from_nhwc(dx), xx.grad)
        dw = torch.zeros(C, 9, device=DEV)
        ops.dwconv_wgrad(ops.to_nhwc(gy), ops.to_nhwc(xx.detach()), dw, N, H, W, C, P, Q, st, 1)
        close(dw, w.grad.reshape(C, 9), 2e-2, 2e-2)


@pytest.mark.parametrize('case', [(8, 96, 16, 16, 1, 4), (8, 144, 15, 15, 2, 2),
                                  (4, 960, 4, 4, 1, 2), (3, 16, 7, 9, 2, 1), (6, 40, 5, 11, 1, 3),
                                  # one group, > 256 blocks: the grid-stride forward
                                  (32, 96, 32, 32, 1, 1), (64, 144, 31, 33, 2, 1)])
def test_depthwise_strips_ghost_stats(case):
    """Strip/sliding-window depthwise kernels: odd widths, stride 2, ghost-BN groups, and
    blocks that straddle two BN groups (tiny images, many channels)."""
    ops = _ops()
    N, C, H, W, st, G = case
    torch.manual_seed(1)
    xx = bf(torch.randn(N, C, H, W, device=DEV)).requires_grad_(True)
    w = torch.randn(C, 1, 3, 3, device=DEV).requires_grad_(True)
    ref = F.conv2d(xx, bf(w), stride=st, padding=1, groups=C)
    P, Q = ref.shape[2:]
    y = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(G, 2, C, device=DEV)
    wf = bf(w.detach()).reshape(C, 9).contiguous()
    ops.dwconv_fwd(ops.to_nhwc(xx.detach()), wf, y, N, H, W, C, P, Q, st, 1, stats=stats,
                   group_rows=(N // G) * P * Q)
    close(ops.from_nhwc(y), ref)
    yr = bf(ref).reshape(G, N // G, C, P, Q)
    close(stats[:, 0], yr.sum((1, 3, 4)), 1e-2, 0.5)
    close(stats[:, 1], yr.pow(2).sum((1, 3, 4)), 1e-2, 0.5)
    gy = bf(torch.randn_like(ref))
    ref.backward(gy)
    dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    ops.dwconv_dgrad(ops.to_nhwc(gy), wf, dx, N, H, W, C, P, Q, st, 1)
    close(ops.from_nhwc(dx), xx.grad)
    dw = torch.zeros(C, 9, device=DEV)
    ops.dwconv_wgrad(ops.to_nhwc(gy), ops.to_nhwc(xx.detach()), dw, N, H, W, C, P, Q, st, 1)
    close(dw, w.grad.reshape(C, 9), 2e-2, 2e-2)
    # column-segmented rows, block partials summed by the reduce kernel (engine path)
    slab = torch.full((ops.dwconv_wgrad_slab_floats(N, P, Q, C),), float('nan'), device=DEV)
    dw2 = torch.zeros(C, 9, device=DEV)
    ops.dwconv_wgrad(ops.to_nhwc(gy), ops.to_nhwc(xx.detach()), dw2, N, H, W, C, P, Q, st, 1,
                     slab=slab)
    close(dw2, w.grad.reshape(C, 9), 2e-2, 2e-2)


def conv_pro_direct(ops, x, wk, out, spec, slab, plan, pro):
    """conv_fwd(pro=...) without the engine's pointwise-only policy (the kernel takes any
    R x S; the policy is a speed choice)."""
    from mercury_amd.ops import conv as cv
    grp = spec.group_rows if spec.group_rows else spec.M
    cv.lib().igemm_pro(cv.ptr(x), cv.ptr(wk), cv.ptr(out), spec.K, 0, 0, spec.K, grp,
                       cv.ptr(slab) if plan[2] > 1 else 0, spec.H, spec.W, spec.Cp, spec.P, spec.Q,
                       spec.R, spec.S, spec.stride, spec.pad, spec.R * spec.S * spec.Cp // 8,
                       spec.K, spec.M, plan[0], plan[1], plan[2], cv.stream_ptr(),
                       *cv._pro_args(pro, spec))


@pytest.mark.parametrize('mode', ['train_keep', 'ghost', 'eval'])
@pytest.mark.parametrize('case', [(8, 16, 16, 64, 64, 3, 3, 1, 1), (4, 8, 8, 128, 256, 1, 1, 1, 0),
                                  (64, 4, 4, 64, 128, 3, 3, 2, 1)])
def test_conv_fwd_bn_apply_prologue(case, mode):
    """conv(act(bn(y))) with the BN-apply + ReLU done in the conv's operand load equals the
    separate bn_apply pass followed by the plain conv, and an fp32 torch reference; in train
    mode the kept activation equals bn_apply's output."""
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, pro_ok, slab_bytes
    N, H, W, C, K, R, S, st, pd = case
    if mode == 'train_keep' and st != 1:
        pytest.skip('keep needs a stride-1 same conv')
    g = torch.Generator(device='cpu').manual_seed(7)
    yb = bf(torch.randn(N, C, H, W, generator=g) * 2 + 0.5).to(DEV)         # producer output
    w = bf(torch.randn(K, C, R, S, generator=g) / math.sqrt(C * R * S)).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.3).to(DEV)
    yn = ops.to_nhwc(yb)
    gimgs = N // 2 if mode == 'ghost' else 0     # two ghost groups
    G = N // gimgs if gimgs else 1
    spec = ConvSpec(N, H, W, C, K, R, S, st, pd)
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    ycnt = (gimgs or N) * H * W
    yg = yb.view(G, -1, C, H, W)
    stats = torch.stack([yg.sum((1, 3, 4)), yg.pow(2).sum((1, 3, 4))], 1).contiguous()  # [G][2][C]
    rmean = (torch.randn(C, generator=g) * 0.2).to(DEV)
    rvar = (torch.rand(C, generator=g) + 0.5).to(DEV)
    # reference activation (fp32 from the bf16 input), then bf16 as the kernels store it
    if mode == 'eval':
        mean = rmean.view(1, 1, C, 1, 1).expand(G, 1, C, 1, 1)
        var = rvar.view(1, 1, C, 1, 1).expand(G, 1, C, 1, 1)
    else:
        mean = (stats[:, 0] / ycnt).view(G, 1, C, 1, 1)
        var = (stats[:, 1] / ycnt).view(G, 1, C, 1, 1) - mean ** 2
    a = torch.relu((yg - mean) / torch.sqrt(var + 1e-5) * gamma.view(1, 1, C, 1, 1)
                   + beta.view(1, 1, C, 1, 1)).view(N, C, H, W)
    ref = F.conv2d(bf(a), w, stride=st, padding=pd)
    plan = fwd_plan(spec)
    if R == 1:
        assert pro_ok(spec, plan, keep=mode == 'train_keep')
    wk, _ = ops.pack_conv_weight(w)
    slab = torch.zeros(max(1, slab_bytes(spec.M, K, *plan[:3]) // 4), device=DEV)
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    keep = torch.full_like(yn, float('nan')) if mode == 'train_keep' else None
    pro = dict(gamma=gamma, beta=beta, act='relu', eps=1e-5, keep=keep)
    if mode == 'eval':
        pro.update(rmean=rmean, rvar=rvar)
    else:
        pro.update(stats=stats.reshape(-1), count=ycnt)
    conv_pro_direct(ops, yn, wk, out, spec, slab, plan, pro)
    got = out.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2)
    close(got, ref)
    # unfused path: bn_apply pass, then the plain conv
    an = torch.empty_like(yn)
    ops.bn_apply(yn, None if mode == 'eval' else stats.reshape(-1), gamma, beta, an, N * H * W, C,
                 group_rows=gimgs * H * W, act='relu',
                 running=(rmean, rvar) if mode == 'eval' else None)
    out2 = torch.empty_like(out)
    ops.conv_fwd(an, wk, out2, spec, slab=slab, plan=plan)
    close(out, out2, rtol=1e-2, atol=1e-2)
    if keep is not None:
        assert not torch.isnan(keep.float()).any()
        close(keep.float(), an.float(), rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('act', ['none', 'relu'])
def test_conv_fwd_bn_residual_prologue(act):
    """The block-final form of the prologue: conv(act(bn(y) + res)) with the residual added in
    the operand load and the block output kept == bn_apply(res mode) then the plain conv."""
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, pro_ok, slab_bytes
    N, H, C, K = 8, 16, 32, 96
    g = torch.Generator(device='cpu').manual_seed(11)
    yb = bf(torch.randn(N, C, H, H, generator=g) * 2 + 0.5).to(DEV)
    rb = bf(torch.randn(N, C, H, H, generator=g)).to(DEV)
    w = bf(torch.randn(K, C, 1, 1, generator=g) / math.sqrt(C)).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.3).to(DEV)
    yn, rn = ops.to_nhwc(yb), ops.to_nhwc(rb)
    spec = ConvSpec(N, H, H, C, K, 1, 1, 1, 0)
    stats = torch.stack([yb.sum((0, 2, 3)), yb.pow(2).sum((0, 2, 3))]).contiguous()
    plan = fwd_plan(spec)
    assert pro_ok(spec, plan, keep=True)
    wk, _ = ops.pack_conv_weight(w)
    slab = torch.zeros(max(1, slab_bytes(spec.M, K, *plan[:3]) // 4), device=DEV)
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    keep = torch.full_like(yn, float('nan'))
    pro = dict(gamma=gamma, beta=beta, act=act, eps=1e-5, keep=keep, res=rn,
               stats=stats.reshape(-1), count=N * H * H)
    ops.conv_fwd(yn, wk, out, spec, slab=slab, plan=plan, pro=pro)
    an = torch.empty_like(yn)
    ops.bn_apply(yn, stats.reshape(-1), gamma, beta, an, N * H * H, C, act=act, res=rn)
    out2 = torch.empty_like(out)
    ops.conv_fwd(an, wk, out2, spec, slab=slab, plan=plan)
    close(out, out2, rtol=1e-2, atol=1e-2)
    assert not torch.isnan(keep.float()).any()
    close(keep.float(), an.float(), rtol=1e-2, atol=1e-2)


def test_fused_bn_paths_propagate_nan_like_bn_hip():
    """act='none' (MobileNetV2's linear bottleneck): a NaN in the producer output must come out
    of the fused prologue as NaN, exactly where the standalone bn_apply + conv produces NaN,
    and the fused dgrad BN-backward reduction must see it (sums NaN, as bn_bwd's)."""
    ops = _ops()
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes, dgrad_plan
    N, H, W, C, K = 4, 8, 8, 64, 128
    spec = ConvSpec(N, H, W, C, K, 1, 1, 1, 0)
    g = torch.Generator(device='cpu').manual_seed(3)
    y = bf(torch.randn(N * H * W, C, generator=g)).to(DEV)
    y[5, 7] = float('nan')
    y[77, 0] = float('nan')
    yn = y.to(torch.bfloat16)
    w = bf(torch.randn(K, C, 1, 1, generator=g) / 8).to(DEV)
    wk, wt = ops.pack_conv_weight(w)
    gamma = torch.ones(C, device=DEV)
    beta = torch.zeros(C, device=DEV)
    rmean, rvar = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
    plan = fwd_plan(spec)
    slab = torch.zeros(max(1, slab_bytes(spec.M, K, *plan[:3]) // 4), device=DEV)
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    conv_pro_direct(ops, yn, wk, out, spec, slab, plan,
                    dict(gamma=gamma, beta=beta, act='none', eps=0.0, rmean=rmean, rvar=rvar))
    an = torch.empty_like(yn)
    ops.bn_apply(yn, None, gamma, beta, an, N * H * W, C, act='none', eps=0.0,
                 running=(rmean, rvar))
    out2 = torch.empty_like(out)
    ops.conv_fwd(an, wk, out2, spec, slab=slab, plan=plan)
    nan1, nan2 = torch.isnan(out.float()), torch.isnan(out2.float())
    assert nan2.any() and torch.equal(nan1, nan2)
    fin = ~nan1
    close(out.float()[fin], out2.float()[fin], rtol=1e-2, atol=1e-2)
    # backward, act none: the fused reduce must pass dz = dx even where the saved activation
    # is NaN (bn_bwd's act_mask is 1 for none), so sum(dz) is the plain column sum of dx
    dspec = ConvSpec(N, H, W, C, K, 1, 1, 1, 0)
    gy = bf(torch.randn(spec.M, K, device=DEV)).to(torch.bfloat16)
    dx = torch.empty(N * H * W, C, dtype=torch.bfloat16, device=DEV)
    yc = bf(torch.randn(N * H * W, C, device=DEV)).to(torch.bfloat16)
    stats = torch.stack([yc.float().sum(0), yc.float().pow(2).sum(0)]).contiguous()
    sums = torch.zeros(ops.sums_numel(C), device=DEV)
    dplan = dgrad_plan(dspec)
    dslab = torch.zeros(max(1, slab_bytes(N * H * W, C, *dplan) // 4), device=DEV)
    ops.conv_dgrad(gy, wt, dx, dspec, slab=dslab, plan=dplan,
                   bw=dict(out=an, y=yc, stats=stats, sums=sums, act='none', eps=1e-5))
    tot = ops.sums_total(sums, C)
    assert torch.isfinite(tot[:2]).all()
    close(tot[0], dx.float().sum(0), 1e-3, 1e-2)


def _halo_case(ops, case, plan, gimgs):
    from mercury_amd.ops.conv import ConvSpec
    N, H, W, C, K, R, S, st, pd = case
    x, w = _mk(case, 5)
    spec = ConvSpec(*case)
    G = N // gimgs if gimgs else 1
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(G, 2, K, device=DEV)
    ops.conv_fwd(ops.to_nhwc(x), ops.pack_conv_weight(w)[0], out, spec, stats=stats, plan=plan)
    ref = F.conv2d(x, w, padding=1)
    close(out.view(N, H, W, K).permute(0, 3, 1, 2), ref)
    rb = bf(ref)
    for gi in range(G):
        r = rb[gi * (gimgs or N):(gi + 1) * (gimgs or N)]
        close(stats[gi, 0], r.sum((0, 2, 3)), rtol=1e-2, atol=0.5)
        close(stats[gi, 1], r.pow(2).sum((0, 2, 3)), rtol=1e-2, atol=0.5)


def test_head_wide_gemm_path_matches_torch():
    """ImageNet-width head (2048 -> 1000): pool kernel + fp32 tiled FC + loss kernel, B not a
    multiple of the 64-row tile; train (IS-weighted, dlogits) and gradnorm score modes."""
    ops = _ops()
    from mercury_amd.importance.pool import classifier_gradnorm
    B, HW, C, K = 70, 49, 2048, 1000
    act = bf(torch.rand(B, HW, C, device=DEV))
    w = torch.randn(K, C, device=DEV) * 0.02
    b = torch.randn(K, device=DEV) * 0.1
    lab = torch.randint(0, K, (B,), device=DEV)
    isw = torch.rand(B, device=DEV) + 0.5
    pooled = torch.empty(B, C, device=DEV)
    logits = torch.empty(B, K, device=DEV)
    dlog = torch.empty(B, K, device=DEV)
    losses = torch.empty(B, device=DEV)
    meters = torch.zeros(8, device=DEV)
    ops.head_fwd(act.to(torch.bfloat16), w, b, lab.int(), B, HW, C, K, 'train', pooled=pooled,
                 logits=logits, dlogits=dlog, losses=losses, isw=isw, meters=meters)
    h = act.double().mean(1)
    ref_logits = h @ w.double().t() + b.double()
    close(pooled, h.float(), rtol=1e-5, atol=1e-6)
    close(logits, ref_logits.float(), rtol=1e-4, atol=1e-4)
    l = F.cross_entropy(ref_logits, lab, reduction='none')
    close(losses, l.float(), rtol=1e-4, atol=1e-4)
    p = torch.softmax(ref_logits, 1) - F.one_hot(lab, K).double()
    close(dlog, (p / (B * isw.double()[:, None])).float(), rtol=1e-3, atol=1e-7)
    assert meters[2].item() == (ref_logits.argmax(1) == lab).sum().item()
    # backward through the wide-head GEMMs vs autograd of the same fp32 graph
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    ar = act.clone().requires_grad_(True)
    (F.cross_entropy(ar.mean(1) @ wr.t() + br, lab, reduction='none') / isw).mean().backward()
    dw, db = torch.empty_like(w), torch.empty_like(b)
    dact = torch.empty(B, HW, C, dtype=torch.bfloat16, device=DEV)
    ops.head_bwd(pooled, dlog, w, dw, db, dact, B, HW, C, K)
    close(dw, wr.grad, rtol=1e-3, atol=1e-7)
    close(db, br.grad, rtol=1e-3, atol=1e-7)
    close(dact, ar.grad, rtol=1e-2, atol=1e-8)
    g = torch.empty(B, device=DEV)
    ops.head_fwd(act.to(torch.bfloat16), w, b, lab.int(), B, HW, C, K, 'score', pooled=pooled,
                 logits=logits, losses=g, score='gradnorm')
    close(g, classifier_gradnorm(ref_logits.float(), lab, h.float()), rtol=1e-4, atol=1e-5)


def test_pool_with_fused_bn_matches_bn_apply_then_pool():
    """Stem max pool applying ghost-group BN + ReLU == bn_apply pass + plain pool, bit for bit
    (same bf16 rounding), from batch sums and from running statistics, negative BN scales
    included (the kernel pools the raw max / min and transforms once)."""
    ops = _ops()
    N, H, W, C, G = 8, 14, 14, 64, 4
    k, st, pd = 3, 2, 1
    P = Q = (H + 2 * pd - k) // st + 1
    y = bf(torch.randn(N, H, W, C, device=DEV)).to(torch.bfloat16).contiguous()
    yf = y.float().view(G, -1, C)
    stats = torch.stack([yf.sum(1), (yf * yf).sum(1)], 1).contiguous()      # [G][2][C]
    gamma = torch.randn(C, device=DEV)            # negative scales take the min branch
    gamma[:8] = -gamma[:8].abs() - 0.1
    beta = torch.randn(C, device=DEV) * 0.2
    rm, rv = torch.randn(C, device=DEV) * 0.1, torch.rand(C, device=DEV) + 0.5
    for bn in (dict(stats=stats, group_imgs=N // G), dict(rmean=rm, rvar=rv)):
        a = torch.empty_like(y)
        if 'stats' in bn:
            ops.bn_apply(y, stats, gamma, beta, a, N * H * W, C, group_rows=(N // G) * H * W,
                         act='relu', eps=1e-5)
        else:
            ops.bn_apply(y, None, gamma, beta, a, N * H * W, C, group_rows=N * H * W,
                         act='relu', eps=1e-5, running=(rm, rv))
        ref = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=DEV)
        ops.pool2d_fwd(a, ref, N, H, W, C, P, Q, k, st, pd, True)
        out = torch.empty_like(ref)
        ops.pool2d_fwd(y, out, N, H, W, C, P, Q, k, st, pd, True,
                       bn=dict(bn, gamma=gamma, beta=beta, act='relu', eps=1e-5))
        assert torch.equal(out, ref)


def test_maxpool_stem_shape_bwd_matches_torch():
    """3x3/s2/p1 pool at an ImageNet-stem-like shape (byte argmax, 8-channel threads)."""
    ops = _ops()
    N, C, H, W = 4, 64, 56, 56
    xx = bf(torch.randn(N, C, H, W, device=DEV)).requires_grad_(True)
    ref = F.max_pool2d(xx, 3, 2, 1)
    P, Q = ref.shape[2:]
    y = torch.empty(N, P, Q, C, dtype=torch.bfloat16, device=DEV)
    am = torch.empty(N * P * Q * C, dtype=torch.uint8, device=DEV)
    ops.pool2d_fwd(ops.to_nhwc(xx.detach()), y, N, H, W, C, P, Q, 3, 2, 1, True, am)
    assert torch.equal(ops.from_nhwc(y).float(), bf(ref.detach()))
    gy = bf(torch.randn_like(ref))
    ref.backward(gy)
    dx = torch.empty(N, H, W, C, dtype=torch.bfloat16, device=DEV)
    ops.maxpool2d_bwd(ops.to_nhwc(gy), am, dx, N, H, W, C, P, Q, 3, 2, 1)
    close(ops.from_nhwc(dx), xx.grad, 1e-2, 1e-2)


@pytest.mark.parametrize('stride', [1, 2])
@pytest.mark.parametrize('ghost', [False, True])
@pytest.mark.parametrize('N', [8, 64])
def test_dwconv_input_bn_prologue_matches_bn_apply_then_dw(stride, ghost, N):
    """Depthwise 3x3 with its input's BN + ReLU6 applied to every loaded chunk (MobileNetV2
    expand -> dw) == bn_apply pass + plain depthwise conv; the kept activation == bn_apply's.
    N = 64 without ghost groups runs the grid-stride (one statistics group) kernel."""
    ops = _ops()
    H, W, C = 16, 16, 96
    P, Q = H // stride, W // stride
    g = torch.Generator(device='cpu').manual_seed(11 + stride)
    y = bf(torch.randn(N * H * W, C, generator=g) * 2 + 0.3).to(DEV).to(torch.bfloat16)
    w = (torch.randn(C, 9, generator=g) * 0.3).to(DEV)
    gamma = (torch.rand(C, generator=g) + 0.5).to(DEV)
    beta = (torch.randn(C, generator=g) * 0.3).to(DEV)
    gi = 4 if ghost else N
    G = N // gi
    yg = y.float().view(G, gi * H * W, C)
    stats = torch.stack([yg.sum(1), yg.pow(2).sum(1)], 1).contiguous().reshape(-1)
    cnt = gi * H * W
    a = torch.empty_like(y)
    ops.bn_apply(y, stats, gamma, beta, a, N * H * W, C, group_rows=cnt if ghost else 0,
                 act='relu6')
    ref = torch.empty(N * P * Q, C, dtype=torch.bfloat16, device=DEV)
    ops.dwconv_fwd(a, w, ref, N, H, W, C, P, Q, stride, 1)
    out = torch.empty_like(ref)
    keep = torch.full_like(y, float('nan'))
    ops.dwconv_fwd(y, w, out, N, H, W, C, P, Q, stride, 1,
                   pro=dict(stats=stats, gamma=gamma, beta=beta, act='relu6', eps=1e-5,
                            count=cnt, group_imgs=gi, keep=keep))
    close(out, ref, rtol=1e-2, atol=1e-2)
    assert not torch.isnan(keep.float()).any()
    close(keep, a, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize('case', [(8, 96, 16, 16, 1, 'relu6'), (8, 144, 15, 15, 2, 'relu6'),
                                  (4, 960, 4, 4, 1, 'relu6'), (6, 40, 5, 11, 1, 'relu'),
                                  (3, 16, 7, 9, 2, 'none')])
def test_dwconv_dgrad_fused_bn_backward_reduce(case):
    """The depthwise dgrad with bw= reduces the feeding BN's backward sums exactly like
    bn_bwd's reduce pass over the same dx (MobileNetV2's expand BN + ReLU6 -> dw conv)."""
    ops = _ops()
    N, C, H, W, st, act = case
    torch.manual_seed(3)
    M = N * H * W
    y = bf(torch.randn(M, C, device=DEV) * 1.5 + 0.3).to(torch.bfloat16)
    yf = y.float()
    stats = torch.stack([yf.sum(0), yf.pow(2).sum(0)]).contiguous()        # [2][C]
    gamma = torch.rand(C, device=DEV) + 0.5
    beta = torch.randn(C, device=DEV) * 0.2
    out = torch.empty_like(y)
    ops.bn_apply(y, stats.reshape(-1), gamma, beta, out, M, C, act=act)
    P, Q = (H - 1) // st + 1, (W - 1) // st + 1
    gy = bf(torch.randn(N, P, Q, C, device=DEV)).to(torch.bfloat16)
    wf = torch.randn(C, 9, device=DEV)
    dx = torch.empty(M, C, dtype=torch.bfloat16, device=DEV)
    ops.dwconv_dgrad(gy, wf, dx, N, H, W, C, P, Q, st, 1)
    dx2 = torch.empty_like(dx)
    sums = torch.zeros(ops.sums_numel(C), device=DEV)
    ops.dwconv_dgrad(gy, wf, dx2, N, H, W, C, P, Q, st, 1,
                     bw=dict(out=out, y=y, stats=stats, sums=sums, act=act, eps=1e-5))
    assert torch.equal(dx, dx2)
    ref = torch.zeros(ops.sums_numel(C), device=DEV)
    scratch = torch.empty_like(y)
    ops.bn_bwd(dx, out, y, stats.reshape(-1), gamma, ref, scratch, M, C, act=act, eps=1e-5)
    close(ops.sums_total(sums, C)[:2], ops.sums_total(ref, C)[:2], 2e-3, 1e-2)


@pytest.mark.parametrize('stride', [1, 2])
@pytest.mark.parametrize('fused', [False, True])
def test_dwconv_bwd_pair_matches_separate(stride, fused):
    """dwconv_bwd (dgrad + slab wgrad in one launch, reduce immediate or deferred to the
    batched reduce) == dwconv_dgrad + dwconv_wgrad, and the wgrad == torch."""
    ops = _ops()
    N, H, C = 8, 16, 96
    P = (H + 2 - 3) // stride + 1
    x = bf(torch.randn(N, C, H, H, device=DEV))
    w = (torch.randn(C, 1, 3, 3, device=DEV) * 0.2)
    gy = bf(torch.randn(N, C, P, P, device=DEV))
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    F.conv2d(xr, wr, stride=stride, padding=1, groups=C).backward(gy)
    xn, gyn = ops.to_nhwc(x), ops.to_nhwc(gy)
    wf = w.view(C, 9).contiguous()
    Mx = N * H * H
    bw = bw2 = None
    if fused:
        y = bf(torch.randn(Mx, C, device=DEV)).to(torch.bfloat16)
        out = bf(torch.relu(torch.randn(Mx, C, device=DEV))).to(torch.bfloat16)
        stats = torch.stack([y.float().sum(0), y.float().pow(2).sum(0)]).contiguous()
        bw = dict(out=out, y=y, stats=stats, sums=torch.zeros(ops.sums_numel(C), device=DEV),
                  act='relu')
        bw2 = dict(bw, sums=torch.zeros(ops.sums_numel(C), device=DEV))
    dx1 = torch.empty(Mx, C, dtype=torch.bfloat16, device=DEV)
    dw1 = torch.zeros(C * 9, device=DEV)
    slab = torch.zeros(ops.dwconv_wgrad_slab_floats(N, P, P, C), device=DEV)
    ops.dwconv_dgrad(gyn, wf, dx1, N, H, H, C, P, P, stride, 1, bw=bw)
    ops.dwconv_wgrad(gyn, xn, dw1, N, H, H, C, P, P, stride, 1, slab=slab)
    for defer in (False, True):
        dx2 = torch.empty_like(dx1)
        dw2 = torch.zeros_like(dw1)
        if bw2 is not None:
            bw2['sums'].zero_()
        ops.dwconv_bwd(gyn, xn, wf, dx2, dw2, N, H, H, C, P, P, stride, 1, slab, bw=bw2,
                       reduce=not defer)
        if defer:
            nblk = ops.dwconv_wgrad_blocks(N, P, P, C)
            ops.dwconv_wgrad_reduce_batch([(slab, dw2, C, nblk)])
        assert torch.equal(dx1, dx2)
        close(dw2, dw1, 1e-4, 1e-4)
        if fused:
            close(ops.sums_total(bw2['sums'], C), ops.sums_total(bw['sums'], C), 1e-4, 1e-3)
    close(dw1.view(C, 3, 3), wr.grad.view(C, 3, 3), 2e-2, 2e-2)
    close(ops.from_nhwc(dx1.view(N, H, H, C), C), xr.grad, 2e-2, 2e-2)


@pytest.mark.parametrize('two', [False, True])
def test_head_bwd_fused_bn_backward_reduce(two):
    """head_bwd(bw=...) reduces the final BN's backward sums from the activation gradient it
    writes (dz = dact * relu'(out)) -- vs torch fp32 on the produced dact."""
    ops = _ops()
    B, HW, C, K = 16, 16, 64, 10
    g = torch.Generator(device='cpu').manual_seed(5)
    pooled = torch.randn(B, C, generator=g).to(DEV)
    dlogits = torch.randn(B, K, generator=g).to(DEV) * 0.1
    w = torch.randn(K, C, generator=g).to(DEV) * 0.1
    dw = torch.zeros(K * C, device=DEV)
    db = torch.zeros(K, device=DEV)
    dact = torch.empty(B * HW * C, dtype=torch.bfloat16, device=DEV)
    Mx = B * HW
    y = bf(torch.randn(Mx, C, generator=g).to(DEV) * 2 + 0.5).to(torch.bfloat16)
    y2 = bf(torch.randn(Mx, C, generator=g).to(DEV)).to(torch.bfloat16)
    out = bf(torch.relu(torch.randn(Mx, C, generator=g).to(DEV))).to(torch.bfloat16)
    stats = torch.stack([y.float().sum(0), y.float().pow(2).sum(0)]).contiguous()
    stats2 = torch.stack([y2.float().sum(0), y2.float().pow(2).sum(0)]).contiguous()
    sums = torch.zeros(ops.sums_numel(C), device=DEV)
    bw = dict(out=out, y=y, stats=stats, sums=sums, act='relu', eps=1e-5)
    if two:
        bw.update(y2=y2, stats2=stats2)
    assert ops.head_bwd(pooled, dlogits, w, dw, db, dact, B, HW, C, K, bw=bw)
    d = dact.float().view(Mx, C)
    close(d.view(B, HW, C)[:, 0], (dlogits @ w) / HW, 1e-2, 1e-3)
    dz = d * (out.float() > 0)

    def xhat(t, s):
        mu = s[0] / Mx
        var = (s[1] / Mx - mu * mu).clamp_min(0)
        return (t.float() - mu) / torch.sqrt(var + 1e-5)
    tot = ops.sums_total(sums, C)
    close(tot[0], dz.sum(0), 1e-3, 1e-2)
    close(tot[1], (dz * xhat(y, stats)).sum(0), 1e-3, 1e-2)
    if two:
        close(tot[2], (dz * xhat(y2, stats2)).sum(0), 1e-3, 1e-2)
