"""Halo-tile conv (csrc/hconv.hip) vs a plain PyTorch fp32 reference.

    out = conv2d(x, w)              (fp32 on the bf16-rounded x and w)

with the output BN sums of the epilogue per ghost-BN image group and split-K over 64-channel
slices (per-tile kernel); the persistent and row-step kernels also take the PRODUCER's
BatchNorm + activation in the halo staging (MODE 1):

    a   = act(bn(y))                 (fp32 from the bf16 tensors, then bf16)
    out = conv2d(a, w)
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def bf(x):
    return x.to(torch.bfloat16).float()


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol + rtol * scale, 'max err %g (scale %g)' % (err, scale)


CASES = [
    # N, H, C, K, R, stride, plan
    (8, 16, 64, 64, 3, 1, (128, 64, 1)),     # TR rows of one image
    (8, 16, 128, 64, 3, 1, (64, 64, 2)),     # split over the two 64-channel slices
    (8, 32, 64, 64, 3, 1, (256, 64, 1)),     # layer1 scoring tile
    (8, 16, 64, 128, 3, 2, (64, 128, 1)),    # stride 2: even/odd column halves
    (8, 8, 128, 128, 3, 1, (128, 128, 1)),   # IMG = 2 whole images per tile
    (16, 4, 128, 128, 3, 1, (64, 128, 2)),   # IMG = 4, split
    (8, 16, 256, 128, 3, 1, (256, 128, 2)),  # 256 x 128 tile, two slices per split block
    (4, 8, 192, 64, 3, 1, (64, 64, 1)),      # three slices in one block (halo prefetch)
    (16, 4, 256, 128, 3, 1, (128, 128, 1)),  # layer4 images: row-term halo swizzle (SWA 6)
    (16, 8, 128, 128, 3, 1, (256, 128, 1)),  # layer3 images, 256-row tile: SWA 6
]


def _bn_ref(y, stats, gamma, beta, cnt, G, running=None, eps=1e-5):
    N, C = y.shape[0], y.shape[1]
    yg = y.view(G, N // G, C, *y.shape[2:])
    if running is not None:
        mean = running[0].view(1, 1, C, 1, 1)
        var = running[1].view(1, 1, C, 1, 1)
    else:
        mean = (stats[:, 0] / cnt).view(G, 1, C, 1, 1)
        var = (stats[:, 1] / cnt).view(G, 1, C, 1, 1) - mean ** 2
    z = (yg - mean) / torch.sqrt(var + eps) * gamma.view(1, 1, C, 1, 1) + beta.view(1, 1, C, 1, 1)
    return z.view_as(y)


@pytest.mark.parametrize('ghost', [False, True])
@pytest.mark.parametrize('case', CASES)
def test_hconv_per_tile(case, ghost):
    """Per-tile plan (splits >= 1): output and (ghost-group) BN sums vs torch fp32."""
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, slab_bytes
    ops.lib()
    N, Hh, C, K, R, st, plan = case
    spec = ConvSpec(N, Hh, Hh, C, K, R, R, st, R // 2)
    gimgs = N // 2 if ghost else 0
    G = 2 if gimgs else 1
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    if H.geometry(spec, plan[0], plan[1], swa=True) is None:
        pytest.skip('tile does not fit')
    g = torch.Generator(device='cpu').manual_seed(11)
    x = bf(torch.randn(N, C, Hh, Hh, generator=g) * 1.5 + 0.3).to(DEV)
    w = bf(torch.randn(K, C, R, R, generator=g) / math.sqrt(C * R * R)).to(DEV)
    ref = F.conv2d(x, w, stride=st, padding=R // 2)
    wk, _ = ops.pack_conv_weight(w)
    out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
    ostats = torch.zeros(G, 2, K, device=DEV)
    slab = torch.zeros(max(1, slab_bytes(spec.M, K, *plan) // 4 + 1), device=DEV)
    H.hconv_fwd(ops.to_nhwc(x), wk, out, spec, plan, stats=ostats, slab=slab)
    torch.cuda.synchronize()
    got = out.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2)
    close(got, ref)
    rg = bf(ref).view(G, -1, K, spec.P, spec.Q)
    close(ostats[:, 0], rg.sum((1, 3, 4)), rtol=1e-2, atol=0.5)
    close(ostats[:, 1], rg.pow(2).sum((1, 3, 4)), rtol=1e-2, atol=0.5)


def test_hconv_matches_igemm_on_scoring_shapes():
    """Plain mode at the B=320 layer shapes (10 ghost groups): same output and BN sums as the
    generic implicit GEMM."""
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    ops.lib()
    for (C, K, Hh, R, st) in [(64, 64, 32, 3, 1), (128, 256, 16, 3, 2), (256, 256, 8, 3, 1),
                              (512, 512, 4, 3, 1), (128, 128, 16, 3, 1)]:
        spec = ConvSpec(320, Hh, Hh, C, K, R, R, st, R // 2)
        spec.group_rows = 32 * spec.P * spec.Q
        plan = H.plan(spec)
        assert plan is not None, (C, K, Hh)
        g = torch.Generator(device='cpu').manual_seed(3)
        x = ops.to_nhwc(bf(torch.randn(320, C, Hh, Hh, generator=g)).to(DEV))
        wk, _ = ops.pack_conv_weight(bf(torch.randn(K, C, R, R, generator=g) * 0.05).to(DEV))
        outs, sts = [], []
        for use_h in (False, True):
            out = torch.empty(spec.M, K, dtype=torch.bfloat16, device=DEV)
            stt = torch.zeros(10, 2, K, device=DEV)
            p = plan if use_h else fwd_plan(spec)
            slab = torch.zeros(max(1, slab_bytes(spec.M, K, *p[:3]) // 4 + 1), device=DEV)
            if use_h:
                H.hconv_fwd(x, wk, out, spec, p, stats=stt, slab=slab)
            else:
                ops.conv_fwd(x, wk, out, spec, stats=stt, slab=slab, plan=p)
            outs.append(out)
            sts.append(stt)
        torch.cuda.synchronize()
        close(outs[1], outs[0], rtol=1e-2, atol=1e-2)
        close(sts[1], sts[0], rtol=1e-3, atol=0.5)


PERSIST_CASES = [
    # N, H, C, K, stride, (bm, bn), ghost images (0: one group)
    (320, 32, 64, 64, 1, (128, 64), 32),     # layer1 scoring shape: 10 tiles per block
    (320, 32, 64, 64, 1, (256, 64), 32),     # 256-row tiles (4 x 1 waves)
    (320, 16, 128, 128, 1, (256, 64), 32),   # IMG = 1, TR = 16, two slices
    (96, 32, 64, 64, 1, (64, 64), 0),        # uneven tiles per block, no ghost groups
    (160, 16, 128, 128, 1, (128, 64), 32),   # two slices per tile, two N tiles
    (128, 32, 64, 128, 2, (64, 64), 32),     # stride 2 (even / odd column halves)
    (320, 8, 256, 256, 1, (128, 64), 32),    # IMG = 2, four slices, four N tiles
    (320, 4, 512, 512, 1, (64, 64), 32),     # IMG = 4, eight slices
    # padded row tiles (no whole-row count fills BM): ResNet-50's 56/28/14/7-wide images
    (16, 56, 64, 64, 1, (128, 64), 8),       # 2 x 56 = 112 of 128 rows
    (16, 56, 64, 64, 1, (256, 64), 8),       # 4 x 56 = 224 of 256
    (16, 28, 128, 128, 1, (128, 64), 8),     # 4 x 28 = 112, two slices, two N tiles
    (16, 28, 64, 64, 1, (64, 64), 8),        # 2 x 28 = 56 of 64
    (16, 14, 256, 256, 1, (128, 64), 8),     # 7 x 14 = 98 of 128
    (16, 7, 512, 512, 1, (128, 64), 8),      # IMG = 2 images of 49 = 98 of 128
    (16, 56, 128, 128, 2, (64, 64), 8),      # stride 2 to 28 wide: 2 x 28 = 56 of 64
]


@pytest.mark.parametrize('with_stats', [True, False, 'bn'])
@pytest.mark.parametrize('case', PERSIST_CASES)
def test_hconv_persistent(case, with_stats):
    """Persistent plan (splits == 0): one block per CU walking a strided tile list as one
    continuous DMA / MFMA pipeline -- output and ghost-BN sums vs torch fp32.  'bn': the input's
    ghost-group BN + ReLU applied in the halo staging (MODE 1)."""
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec
    ops.lib()
    N, Hh, C, K, st, (bm, bn), gimgs = case
    spec = ConvSpec(N, Hh, Hh, C, K, 3, 3, st, 1)
    G = N // gimgs if gimgs else 1
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    geo = H.geometry(spec, bm, bn, pad=True)
    assert geo is not None and H.lds_bytes(geo, bm, bn, 0) <= H.LDS_MAX
    assert H.persistent_ok(spec, bm, bn, stats=with_stats)
    padded = geo['IMG'] * geo['TR'] * geo['Q'] < bm
    # padded tiles also run on this launch's own grid (the plan's 4th element, PGRID)
    plan = (bm, bn, 0, 256) if padded else (bm, bn, 0)
    g = torch.Generator(device='cpu').manual_seed(5)
    x = bf(torch.randn(N, C, Hh, Hh, generator=g) * 1.5 + 0.3)
    w = bf(torch.randn(K, C, 3, 3, generator=g) / math.sqrt(C * 9))
    pro, a = None, x
    if with_stats == 'bn':
        gi = gimgs or N
        cnt = gi * Hh * Hh
        xg = x.view(N // gi, gi, C, Hh, Hh)
        st_in = torch.stack([xg.sum((1, 3, 4)), xg.pow(2).sum((1, 3, 4))], 1).contiguous()
        gamma = torch.rand(C, generator=g) + 0.5
        beta = torch.randn(C, generator=g) * 0.3
        a = bf(torch.relu(_bn_ref(x, st_in, gamma, beta, cnt, N // gi)))
        pro = dict(stats=st_in.reshape(-1).to(DEV), gamma=gamma.to(DEV), beta=beta.to(DEV),
                   act='relu', eps=1e-5, count=cnt, group_imgs=gi)
    if pro is not None and H.lds_bytes(geo, bm, bn, 0) + H.persist_table_bytes(spec, pro) > \
            H.LDS_MAX:
        pytest.skip('BN table does not fit beside this tile')
    ref = F.conv2d(a, w, stride=st, padding=1)
    wk, _ = ops.pack_conv_weight(w.to(DEV))
    out = torch.full((spec.M, K), float('nan'), dtype=torch.bfloat16, device=DEV)
    ostats = torch.zeros(G, 2, K, device=DEV) if with_stats else None
    H.hconv_fwd(ops.to_nhwc(x.to(DEV)), wk, out, spec, plan, stats=ostats, pro=pro)
    torch.cuda.synchronize()
    if (bm, bn) == (128, 64) and H.persist_waves() == 8:
        # the 4 x 2 wave layout of the same tile (EngineOptions.hconv_persist_wm8) must agree
        out2 = torch.full_like(out, float('nan'))
        ost2 = torch.zeros_like(ostats) if ostats is not None else None
        ops.lib().hconv_configure(H._CFG['grid'], 8, 4)
        try:
            H.hconv_fwd(ops.to_nhwc(x.to(DEV)), wk, out2, spec, plan, stats=ost2, pro=pro)
            torch.cuda.synchronize()
        finally:
            ops.lib().hconv_configure(H._CFG['grid'], H.persist_waves(), H._CFG['wm8'])
        close(out2.float(), out.float(), rtol=1e-2, atol=1e-2)
        if ostats is not None:
            close(ost2, ostats, rtol=1e-3, atol=0.5)
    got = out.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2).float().cpu()
    assert not torch.isnan(got).any()
    close(got, ref)
    if with_stats:
        rg = bf(ref).view(G, -1, K, spec.P, spec.Q)
        close(ostats[:, 0].cpu(), rg.sum((1, 3, 4)), rtol=1e-2, atol=0.5)
        close(ostats[:, 1].cpu(), rg.pow(2).sum((1, 3, 4)), rtol=1e-2, atol=0.5)


ROW_CASES = [
    # N, H, C, K, (bm, bn), splits (-1), ghost images (0: one group)
    (320, 32, 64, 64, (256, 64), -1, 32),    # layer1 scoring: weight-stationary, 160 KiB LDS
    (64, 32, 64, 64, (256, 64), -1, 0),      # stationary, no ghost groups, uneven tiles/block
    (320, 16, 128, 128, (256, 64), -1, 32),  # layer2: two slices, two channel tiles (streamed)
    (96, 16, 192, 128, (256, 64), -1, 0),    # three slices, uneven tiles per block
    (64, 32, 64, 128, (256, 64), -1, 32),    # C = 64 but two channel tiles: streamed
]


@pytest.mark.parametrize('with_stats', [True, False, 'bn', 'bn_eval', 'bn_grid4'])
@pytest.mark.parametrize('case', ROW_CASES)
def test_hconv_row_step(case, with_stats):
    """Row-step persistent plan (splits < 0, csrc/hconv.hip hrow_kernel): one filter row per
    pipeline step, weights stationary in LDS when C = K = 64 -- output and ghost-BN sums vs
    torch fp32, and the output bit-identical to the persistent kernel's (same MFMA order per
    output: every tap's two 32-deep halves in the same sequence).  'bn' / 'bn_eval': the input's
    BN from the per-block LDS coefficient table (MODE 2); 'bn_grid4': a 4-block grid, so a
    block's tile range spans more than two ghost-BN groups and the kernel loads the statistics
    per slice instead (MODE 1)."""
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec
    ops.lib()
    grid4 = with_stats == 'bn_grid4'
    if grid4:
        if not case[-1]:
            pytest.skip('one statistics group: the table always fits')
        with_stats = 'bn'
    N, Hh, C, K, (bm, bn), splits, gimgs = case
    spec = ConvSpec(N, Hh, Hh, C, K, 3, 3, 1, 1)
    G = N // gimgs if gimgs else 1
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    geo = H.geometry(spec, bm, bn)
    assert geo is not None and H.row_lds_bytes(geo, bm, bn, splits) <= H.LDS_MAX
    assert H.row_ok(spec, bm, bn, stats=with_stats)
    g = torch.Generator(device='cpu').manual_seed(7)
    x = bf(torch.randn(N, C, Hh, Hh, generator=g) * 1.5 + 0.3)
    w = bf(torch.randn(K, C, 3, 3, generator=g) / math.sqrt(C * 9))
    pro, a = None, x
    if with_stats in ('bn', 'bn_eval'):
        # MODE 1: the input's BN (ghost-group batch or running statistics) + ReLU in the halo
        gi = gimgs or N
        cnt = gi * Hh * Hh
        xg = x.view(N // gi, gi, C, Hh, Hh)
        st_in = torch.stack([xg.sum((1, 3, 4)), xg.pow(2).sum((1, 3, 4))], 1).contiguous()
        gamma = torch.rand(C, generator=g) + 0.5
        beta = torch.randn(C, generator=g) * 0.3
        pro = dict(gamma=gamma.to(DEV), beta=beta.to(DEV), act='relu', eps=1e-5, count=cnt,
                   group_imgs=gi)
        if with_stats == 'bn':
            a = bf(torch.relu(_bn_ref(x, st_in, gamma, beta, cnt, N // gi)))
            pro['stats'] = st_in.reshape(-1).to(DEV)
        else:
            run = (torch.randn(C, generator=g) * 0.2, torch.rand(C, generator=g) + 0.5)
            a = bf(torch.relu(_bn_ref(x, None, gamma, beta, cnt, 1, running=run)))
            pro.update(rmean=run[0].to(DEV), rvar=run[1].to(DEV))
    ref = F.conv2d(a, w, padding=1)
    wk, _ = ops.pack_conv_weight(w.to(DEV))
    xn = ops.to_nhwc(x.to(DEV))
    out = torch.full((spec.M, K), float('nan'), dtype=torch.bfloat16, device=DEV)
    ostats = torch.zeros(G, 2, K, device=DEV) if with_stats else None
    if grid4:
        ops.lib().hconv_configure(4, H.persist_waves(), H._CFG['wm8'])
    try:
        H.hconv_fwd(xn, wk, out, spec, (bm, bn, splits), stats=ostats, pro=pro)
        torch.cuda.synchronize()
    finally:
        if grid4:
            ops.lib().hconv_configure(H._CFG['grid'], H.persist_waves(), H._CFG['wm8'])
    got = out.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2).float().cpu()
    assert not torch.isnan(got).any()
    close(got, ref)
    if with_stats:
        rg = bf(ref).view(G, -1, K, spec.P, spec.Q)
        close(ostats[:, 0].cpu(), rg.sum((1, 3, 4)), rtol=1e-2, atol=0.5)
        close(ostats[:, 1].cpu(), rg.pow(2).sum((1, 3, 4)), rtol=1e-2, atol=0.5)
    if pro is None and H.persistent_ok(spec, bm, bn, stats=with_stats) and \
            H.lds_bytes(geo, bm, bn, 0) <= H.LDS_MAX:
        out2 = torch.empty_like(out)
        H.hconv_fwd(xn, wk, out2, spec, (bm, bn, 0), stats=None)
        torch.cuda.synchronize()
        assert torch.equal(out2, out)
