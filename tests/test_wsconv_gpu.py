"""Weight-stationary persistent halo conv (csrc/wsconv.hip) vs a plain PyTorch fp32 reference.

out = conv2d(x, w) (fp32 on the bf16 inputs) for the two instantiated geometries -- ResNet-18's
stride-1 layer1 (32x32, 64 -> 64) and layer2 (16x16, 128 -> 128) convs -- at the scoring batch
with ghost-BN statistics per 32-image group (one block walks several groups: the running sums
must flush at every group edge), at the train batch (one group), with several N tiles, and with
grids that leave blocks without tiles or give them ranges straddling groups.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def bf(x):
    return x.to(torch.bfloat16).float()


CASES = [
    # N, H, C, K, group images (0: whole batch), grid
    (320, 32, 64, 64, 32, 128),
    (32, 32, 64, 64, 0, 128),
    (64, 32, 64, 128, 32, 96),      # two N tiles (each block holds one 64-column weight slice)
    (320, 16, 128, 128, 32, 128),
    (32, 16, 128, 128, 0, 128),
    (48, 16, 128, 256, 16, 60),     # two N tiles of 128, uneven ranges
    (8, 32, 64, 64, 0, 256),        # more blocks than tiles
]


@pytest.mark.parametrize('case', CASES)
def test_wsconv_matches_torch(case):
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec
    ops.lib()
    N, Hh, C, K, gi, grid = case
    spec = ConvSpec(N, Hh, Hh, C, K, 3, 3, 1, 1)
    if gi:
        spec.group_rows = gi * Hh * Hh
    assert H.wsconv_ok(spec), spec
    g = torch.Generator(device='cpu').manual_seed(5 + N + C + K)
    x = bf(torch.randn(N, C, Hh, Hh, generator=g)).to(DEV)
    w = bf(torch.randn(K, C, 3, 3, generator=g) / math.sqrt(C * 9)).to(DEV)
    xn = ops.to_nhwc(x)
    wk, _ = ops.pack_conv_weight(w)
    G = N // gi if gi else 1
    out = torch.empty(N * Hh * Hh * K, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(G * 2 * K, device=DEV)
    H.wsconv_fwd(xn, wk, out, spec, stats=stats, grid=grid)
    torch.cuda.synchronize()
    ref = F.conv2d(x, w, padding=1)                                  # [N][K][H][W] fp32
    got = out.view(N, Hh, Hh, K).permute(0, 3, 1, 2).float()
    err = (got - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-2, err
    # statistics of the bf16-rounded output, per group
    ob = got.reshape(G, N // G, K, Hh, Hh)
    s_ref = ob.sum(dim=(1, 3, 4))
    ss_ref = (ob * ob).sum(dim=(1, 3, 4))
    st = stats.view(G, 2, K)
    torch.testing.assert_close(st[:, 0], s_ref, rtol=1e-3, atol=1e-1)
    torch.testing.assert_close(st[:, 1], ss_ref, rtol=1e-3, atol=1e-1)
    # no statistics: same output
    out2 = torch.empty_like(out)
    H.wsconv_fwd(xn, wk, out2, spec, stats=None, grid=grid)
    torch.cuda.synchronize()
    assert torch.equal(out2, out)


def test_wsconv_engine_plans():
    """EngineOptions.wsconv='score' puts ResNet-18's stride-1 64 / 128-channel scoring convs on
    wsconv (off by default: the scoring-pass A/B measured 1.395 vs 1.3675 ms/step,
    profiles/r4/ab_wsconv.json), and the default engine has none."""
    from mercury_amd.config import EngineOptions
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    import numpy as np
    rng = np.random.RandomState(0)
    x = rng.randint(0, 256, (640, 32, 32, 3), dtype=np.uint8)
    y = rng.randint(0, 10, 640)
    torch.manual_seed(0)
    eng = NativeEngine(ResNet18(10).to(DEV), DEV, 32, 10, opts=EngineOptions(wsconv='score'))
    eng.set_shard(x, y)
    ws = [k[0] for k in eng.score_mode.plan if k[1] == 'wsconv']
    assert len(ws) == 7, ws          # layer1: 4 convs, layer2: 3 stride-1 convs
    assert not any(k[1] == 'wsconv' for k in eng.train_mode.plan)
    eng0 = NativeEngine(ResNet18(10).to(DEV), DEV, 32, 10, opts=EngineOptions())
    eng0.set_shard(x, y)
    assert not any(k[1] == 'wsconv' for k in eng0.score_mode.plan)
