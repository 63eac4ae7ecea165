"""ResNet-50/224 in the engine with its stride-1 3x3 convs on the persistent halo kernel's
PADDED row tiles (``ops.hconv.MEASURED_PAD``: 2 x 56 / 4 x 28 / 7 x 14 rows or 2 x 49-pixel
images per 128- / 256-row tile, the rest of the tile dropped).  The measured table is keyed by
the preset batches (1280 scoring / 128 train); here it is patched to the test batches (320 / 32)
so the same plans run:

* train: the IS-weighted gradients vs torch fp32, bounded by torch-bf16's own error (the
  check of ``test_native_gpu.test_train_forward_backward_matches_torch``);
* scoring: layer1's intra-block BN + ReLU folded into the padded halo staging (MODE 1), losses
  vs the same engine without the padded plans, and both vs ten separate torch forwards.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _patch(monkeypatch, N, fold):
    from mercury_amd.ops import hconv as H
    monkeypatch.setitem(H.MEASURED_PAD, (N, 56, 64, 64), ((256, 64, 0, 256), fold))
    monkeypatch.setitem(H.MEASURED_PAD, (N, 28, 128, 128), ((128, 64, 0, 256), False))
    monkeypatch.setitem(H.MEASURED_PAD, (N, 14, 256, 256), ((256, 64, 0, 256), False))
    monkeypatch.setitem(H.MEASURED_PAD, (N, 7, 512, 512), ((256, 64, 0, 256), False))


def _padded_units(mode):
    return sorted({k[0] for k, p in mode.plan.items()
                   if k[1] in ("hconv", "hconv_bn") and len(p) > 3 and p[2] == 0})


def test_train_gradients_with_padded_halo_plans(monkeypatch):
    from test_native_gpu import test_train_forward_backward_matches_torch
    from mercury_amd.engine import native
    _patch(monkeypatch, 32, False)
    built = []
    orig = native.NativeEngine.set_shard

    def spy(self, *a, **k):
        orig(self, *a, **k)
        built.append(self)
    monkeypatch.setattr(native.NativeEngine, 'set_shard', spy)
    test_train_forward_backward_matches_torch('resnet50_imagenet', 224)
    units = _padded_units(built[-1].train_mode)
    # 3 + 3 + 5 + 2 stride-1 3x3 convs (each stage's first block downsamples in its 3x3)
    assert len(units) == 13, units


def test_scoring_with_padded_halo_plans_and_folded_bn(monkeypatch):
    from mercury_amd import ops
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    torch.manual_seed(2)
    net = build_model('resnet50_imagenet', 10).to(DEV)
    rng = np.random.RandomState(0)
    imgs = rng.randint(0, 256, (400, 224, 224, 3), dtype=np.uint8)
    labels = rng.randint(0, 10, 400)
    losses = {}
    for pad in (False, True):
        with monkeypatch.context() as mp:
            if pad:
                _patch(mp, 320, True)
            else:
                mp.setenv('MERCURY_ENGINE_OPTS', 'hconv_pad=0')
            eng = NativeEngine(net, DEV, batch_size=32, pool_batches=10, use_graphs=False,
                               image_hw=(224, 224))
            eng.set_shard(imgs, labels)
            sm = eng.score_mode
            units = _padded_units(sm)
            if pad:
                assert len(units) == 13, units
                folded = [k[0] for k, p in sm.plan.items() if k[1] == 'hconv_bn' and len(p) > 3]
                assert len(folded) == 3, folded          # layer1's three 3x3 convs
            else:
                assert not units
            sm.stats_arena.zero_()
            if not pad:
                ops.pool_build(eng.shard, eng.shard_labels, eng.ctrl, sm.input, sm.label,
                               sm.index, 320, 32, eng.seed)
                pool, lab = sm.input.clone(), sm.label.clone()
            else:                                        # the same pool in both engines
                sm.input.copy_(pool)
                sm.label.copy_(lab)
            x = eng.forward(sm)
            eng.head(sm, x, 'score')
            torch.cuda.synchronize()
            losses[pad] = sm.losses.clone()
            eng.close()
    data = pool[..., :3].permute(0, 3, 1, 2).float()
    lab = lab.long()
    # the padded plans change only the conv algorithm (and where the layer1 BN is applied):
    # the same losses up to bf16 rounding, amplified through 16 blocks
    a, b = losses[True].double(), losses[False].double()
    cos = float((a @ b) / (a.norm() * b.norm()))
    print('padded vs igemm engine: cos %.6f, mean |diff| %.5f, mean diff %.5f'
          % (cos, (a - b).abs().mean().item(), (a - b).mean().item()))
    assert cos > 0.9995, cos
    # both against ten separate train-mode torch forwards
    ref = []
    net.train()
    with torch.no_grad():
        for j in range(10):
            o = net(data[j * 32:(j + 1) * 32])
            ref.append(F.cross_entropy(o, lab[j * 32:(j + 1) * 32], reduction='none'))
    ref = torch.cat(ref).double()
    err_pad = (a - ref).abs().mean().item()
    err_base = (b - ref).abs().mean().item()
    bias_pad = (a - ref).mean().item()
    bias_base = (b - ref).mean().item()
    print('scoring vs fp32: mean |err| padded %.5f, igemm %.5f; bias padded %.5f, igemm %.5f'
          % (err_pad, err_base, bias_pad, bias_base))
    assert err_pad <= max(1.5 * err_base, 0.01), (err_pad, err_base)
    assert abs(bias_pad) <= max(2.5 * abs(bias_base), 0.01), (bias_pad, bias_base)
