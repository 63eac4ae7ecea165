"""Persistent pointwise GEMM (csrc/pgemm.hip) vs fp32 torch: the 1x1 convs of ResNet-50's
bottlenecks and MobileNetV2's expand / project layers (`pytorch_model.py:44-49`).  Covers every
tile width, odd channel counts (K, N not multiples of 32 / 64), M not a tile multiple, stride-2
row gathers, ghost-BN statistics with groups that straddle tiles, and more tiles than blocks
(the persistent step stream crossing tile boundaries)."""
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
    # N, H, W, C, K, stride, group_imgs, bn, grid
    (32, 16, 16, 256, 64, 1, 0, 64, 0),
    (32, 16, 16, 64, 256, 1, 0, 256, 0),
    (16, 14, 14, 512, 128, 1, 4, 128, 0),      # 784-row groups: tiles straddle group edges
    (8, 28, 28, 128, 512, 2, 0, 256, 0),       # stride-2 shortcut gather
    (20, 8, 8, 96, 24, 1, 0, 64, 0),           # MobileNetV2 project: N = 24, K = 96
    (20, 8, 8, 24, 144, 1, 5, 128, 0),         # expand: K = 24 (< one 32-deep step)
    (12, 9, 11, 40, 72, 1, 0, 64, 7),          # M = 1188 (not a tile multiple), 7 blocks
    (64, 7, 7, 2048, 512, 1, 32, 256, 5),      # deep K, few blocks: long step streams
]


@pytest.mark.parametrize('case', CASES)
def test_pgemm_matches_torch(case):
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec
    ops.lib()
    N, H, W, C, K, st, gimgs, bn, grid = case
    g = torch.Generator(device='cpu').manual_seed(hash(case) % 1000)
    x = bf(torch.randn(N, C, H, W, generator=g)).to(DEV)
    w = bf(torch.randn(K, C, 1, 1, generator=g) / math.sqrt(C)).to(DEV)
    spec = ConvSpec(N, H, W, C, K, 1, 1, st, 0)
    G = N // gimgs if gimgs else 1
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    xn = ops.to_nhwc(x)
    wk, _ = ops.pack_conv_weight(w)
    out = torch.full((spec.M, K), float('nan'), dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(G, 2, K, device=DEV)
    ops.pgemm_fwd(xn, wk, out, spec, stats=stats, bn=bn, grid=grid)
    ref = F.conv2d(x, w, stride=st)
    got = out.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2)
    assert not torch.isnan(got.float()).any()
    close(got, ref)
    rb = bf(ref)
    per = gimgs or N
    for gi in range(G):
        r = rb[gi * per:(gi + 1) * per]
        close(stats[gi, 0], r.sum((0, 2, 3)), rtol=1e-2, atol=0.5)
        close(stats[gi, 1], r.pow(2).sum((0, 2, 3)), rtol=1e-2, atol=0.5)
    # no stats: plain GEMM path, bitwise equal output
    out2 = torch.empty_like(out)
    ops.pgemm_fwd(xn, wk, out2, spec, bn=bn, grid=grid)
    assert torch.equal(out2, out)
