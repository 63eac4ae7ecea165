"""Two forward convs in one launch (ops.conv_fwd_dual, csrc/igemm.hip igemm_dual_kernel): the
downsampling block's 3x3 stride-2 conv and its 1x1 stride-2 shortcut, at the ResNet-18 train and
scoring shapes, against the same convs launched separately (conv_fwd) and against an fp32 torch
conv.  Outputs must be bit-identical to the separate launches (same kernel body per problem)
where K is not split; the ghost-BN sums agree to fp32 rounding (atomic order)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = 'cuda'


@pytest.mark.parametrize('N,H,C,K,groups', [(32, 32, 64, 128, 1), (32, 16, 128, 256, 1),
                                             (32, 8, 256, 512, 1), (320, 32, 64, 128, 10)])
def test_dual_forward_matches_separate(N, H, C, K, groups):
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    torch.manual_seed(0)
    s1 = ConvSpec(N, H, H, C, K, 3, 3, 2, 1)
    s2 = ConvSpec(N, H, H, C, K, 1, 1, 2, 0)
    if groups > 1:
        for s in (s1, s2):
            s.group_rows = s.M // groups
    x = ops.to_nhwc(torch.randn(N, C, H, H, device=DEV))
    w1f = torch.randn(K, C, 3, 3, device=DEV) * 0.05
    w2f = torch.randn(K, C, 1, 1, device=DEV) * 0.1
    w1, _ = ops.pack_conv_weight(w1f)
    w2, _ = ops.pack_conv_weight(w2f)
    p1, p2 = fwd_plan(s1), fwd_plan(s2)
    p2 = (p1[0], p1[1], p2[2])            # same tile shape (the dual kernel's contract)
    slab1 = torch.zeros(max(1, slab_bytes(s1.M, K, *p1[:3]) // 4 + 1), device=DEV)
    slab2 = torch.zeros(max(1, slab_bytes(s2.M, K, *p2[:3]) // 4 + 1), device=DEV)
    outs = []
    for dual in (False, True):
        y1 = torch.empty(s1.M * K, dtype=torch.bfloat16, device=DEV)
        y2 = torch.empty(s2.M * K, dtype=torch.bfloat16, device=DEV)
        st1 = torch.zeros(groups * 2 * K, device=DEV)
        st2 = torch.zeros(groups * 2 * K, device=DEV)
        if dual:
            ok = ops.conv_fwd_dual(dict(x=x, w=w1, out=y1, spec=s1, stats=st1, slab=slab1, plan=p1),
                                   dict(x=x, w=w2, out=y2, spec=s2, stats=st2, slab=slab2, plan=p2))
            assert ok
        else:
            ops.conv_fwd(x, w1, y1, s1, stats=st1, slab=slab1, plan=p1)
            ops.conv_fwd(x, w2, y2, s2, stats=st2, slab=slab2, plan=p2)
        torch.cuda.synchronize()
        outs.append((y1, y2, st1, st2))
    (a1, a2, sa1, sa2), (b1, b2, sb1, sb2) = outs
    # unsplit tiles are bit-identical; split-K tiles are summed by whichever slice arrives last,
    # so their fp32 order (and a bf16 rounding now and then) varies from launch to launch
    for a, b, p in ((a1, b1, p1), (a2, b2, p2)):
        if p[2] == 1:
            assert torch.equal(a, b)
        else:
            torch.testing.assert_close(b.float(), a.float(), rtol=1e-2, atol=1e-2)
    # (the statistics are sums over the bf16 outputs: an output rounded the other way on a
    # split-K tile moves them by ~1 bf16 ulp of that element)
    for sa, sb, p in ((sa1, sb1, p1), (sa2, sb2, p2)):
        torch.testing.assert_close(sb, sa, rtol=1e-4 if p[2] == 1 else 1e-3,
                                   atol=1e-3 if p[2] == 1 else 0.1)
    # and against fp32 torch
    xf = x[..., :C].permute(0, 3, 1, 2).float()
    r1 = torch.nn.functional.conv2d(xf, w1f, stride=2, padding=1).permute(0, 2, 3, 1).reshape(-1, K)
    r2 = torch.nn.functional.conv2d(xf, w2f, stride=2).permute(0, 2, 3, 1).reshape(-1, K)
    torch.testing.assert_close(b1.view(-1, K).float(), r1, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(b2.view(-1, K).float(), r2, rtol=2e-2, atol=2e-2)


def test_dual_forward_refuses_shared_split_slab():
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec
    s1 = ConvSpec(32, 8, 8, 256, 512, 3, 3, 2, 1)
    s2 = ConvSpec(32, 8, 8, 256, 512, 1, 1, 2, 0)
    x = torch.zeros(32, 8, 8, 256, dtype=torch.bfloat16, device=DEV)
    w1 = torch.zeros(512 * 9 * 256, dtype=torch.bfloat16, device=DEV)
    w2 = torch.zeros(512 * 256, dtype=torch.bfloat16, device=DEV)
    slab = torch.zeros(1 << 20, device=DEV)
    y1 = torch.empty(s1.M * 512, dtype=torch.bfloat16, device=DEV)
    y2 = torch.empty(s2.M * 512, dtype=torch.bfloat16, device=DEV)
    assert not ops.conv_fwd_dual(dict(x=x, w=w1, out=y1, spec=s1, slab=slab, plan=(64, 128, 4)),
                                 dict(x=x, w=w2, out=y2, spec=s2, slab=slab, plan=(64, 128, 2)))


@pytest.mark.parametrize('N,H,C,K', [(32, 32, 64, 128), (32, 16, 128, 256), (32, 8, 256, 512)])
def test_shortcut_backward_merged_matches_separate(N, H, C, K):
    """ops.conv.conv_bwd_sc: the block's last conv (3x3 stride 1, K -> K at H/2) backward pair
    and the 1x1 stride-2 shortcut's (C -> K) in one launch vs the two conv_bwd launches."""
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, conv_bwd_sc, dgrad_plan, wgrad_plan, slab_bytes
    torch.manual_seed(0)
    h = H // 2
    s2 = ConvSpec(N, h, h, K, K, 3, 3, 1, 1)          # last conv of the block
    ss = ConvSpec(N, H, H, C, K, 1, 1, 2, 0)          # shortcut
    dy2 = (torch.randn(s2.M, K, device=DEV) * 0.1).to(torch.bfloat16)
    dys = (torch.randn(ss.M, K, device=DEV) * 0.1).to(torch.bfloat16)
    x2 = torch.randn(N, h, h, K, device=DEV).to(torch.bfloat16)
    xs = torch.randn(N, H, H, C, device=DEV).to(torch.bfloat16)
    _, wt2 = ops.pack_conv_weight(torch.randn(K, K, 3, 3, device=DEV) * 0.05)
    _, wts = ops.pack_conv_weight(torch.randn(K, C, 1, 1, device=DEV) * 0.1)
    dp, wp = dgrad_plan(s2), wgrad_plan(s2)
    if tuple(dp[:2]) != (64, 64):
        dp = (64, 64, dp[2])
    wps = wgrad_plan(ss)
    if tuple(wps[:2]) != (64, 64):
        wps = (64, 64, wps[2])
    slab = torch.zeros(max(1, slab_bytes(N * h * h, K, *dp[:3]) // 4 + 1), device=DEV)
    res = []
    for merged in (False, True):
        dx2 = torch.empty(N * h * h * K, dtype=torch.bfloat16, device=DEV)
        dxs = torch.empty(N * H * H * C, dtype=torch.bfloat16, device=DEV)
        dw2 = torch.zeros(K * 9 * K, device=DEV)
        dws = torch.zeros(K * C, device=DEV)
        if merged:
            ok = conv_bwd_sc(dict(dy=dy2, wt=wt2, dx=dx2, x=x2, dw=dw2, spec=s2, dplan=dp, wplan=wp,
                                  slab=slab),
                             dict(dy=dys, wt=wts, dx=dxs, x=xs, dw=dws, spec=ss, wplan=wps))
            assert ok
        else:
            ops.conv_bwd(dys, wts, dxs, xs, dws, ss, wplan=wps)
            ops.conv_bwd(dy2, wt2, dx2, x2, dw2, s2, dplan=dp, wplan=wp, slab=slab)
        torch.cuda.synchronize()
        res.append((dx2, dxs, dw2, dws))
    for a, b in zip(*res):
        torch.testing.assert_close(b.float(), a.float(), rtol=1e-2, atol=1e-2)
