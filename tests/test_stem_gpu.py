"""Dense-k stem conv (csrc/stem.hip) vs fp32 torch: CIFAR 3x3 3->64 (`pytorch_model.py:72`),
ImageNet 7x7/2 3->64 (`:89`), MobileNetV2's 3x3 3->32, the speech VGG's 3x3 1->64 with bias on a
101x161 spectrogram (edge tiles), ghost-BN sums per image group."""
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
    # N, H, W, C, K, R, stride, pad, group_imgs, bias
    (8, 32, 32, 3, 64, 3, 1, 1, 2, False),       # CIFAR ResNet stem, 4 ghost groups
    (6, 32, 32, 3, 32, 3, 1, 1, 0, False),       # MobileNetV2 (CIFAR)
    (3, 224, 224, 3, 64, 7, 2, 3, 1, False),     # ImageNet ResNet 7x7/2
    (4, 101, 161, 1, 64, 3, 1, 1, 2, True),      # speech VGG: 1 channel, bias, edge tiles
    (5, 30, 34, 3, 32, 3, 2, 1, 0, False),       # MobileNetV2 (ImageNet-style) 3x3/2
    (300, 32, 32, 3, 64, 3, 1, 1, 30, False),    # >1 tile per block (the scoring batch path)
]


@pytest.mark.parametrize('case', CASES)
def test_stem_matches_torch(case):
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec
    ops.lib()
    N, H, W, C, K, R, st, pad, gimgs, has_bias = case
    g = torch.Generator(device='cpu').manual_seed(N * 7 + K + R)
    x = bf(torch.randn(N, C, H, W, generator=g)).to(DEV)
    w = bf(torch.randn(K, C, R, R, generator=g) / math.sqrt(C * R * R)).to(DEV)
    bias = (torch.randn(K, generator=g) * 0.1).to(DEV) if has_bias else None
    spec = ConvSpec(N, H, W, C, K, R, R, st, pad)
    G = N // gimgs if gimgs else 1
    if gimgs:
        spec.group_rows = gimgs * spec.P * spec.Q
    xn = ops.to_nhwc(x)
    assert xn.shape[-1] == 8
    wk, _ = ops.pack_conv_weight(w)
    y = torch.full((spec.M, K), float('nan'), dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(G, 2, K, device=DEV)
    ops.stem_fwd(xn, wk, y, spec, stats=stats, bias=bias)
    ref = F.conv2d(x, w, bias, stride=st, padding=pad)
    got = y.view(N, spec.P, spec.Q, K).permute(0, 3, 1, 2)
    assert not torch.isnan(got.float()).any()
    close(got, ref)
    rb = got.float()
    per = gimgs or N
    for gi in range(G):
        r = rb[gi * per:(gi + 1) * per]
        close(stats[gi, 0], r.sum((0, 2, 3)), rtol=1e-3, atol=0.5)
        close(stats[gi, 1], r.pow(2).sum((0, 2, 3)), rtol=1e-3, atol=0.5)
    # no statistics: same output
    y2 = torch.empty_like(y)
    ops.stem_fwd(xn, wk, y2, spec, bias=bias)
    assert torch.equal(y2, y)
