"""CPU checks of the native engine's lowering (module tree -> units, flat layout)."""
import pytest

from mercury_amd.engine.lower import lower, supports
from mercury_amd.models import MobileNetV2, ResNet18, ResNet50, ResNet50_ImageNet, VGG


def test_resnet18_lowering():
    net = ResNet18(10)
    lw = lower(net)
    assert len(lw.blocks) == 1 + 8
    assert sum(1 for b in lw.blocks if b.shortcut is not None) == 3
    assert sum(1 for b in lw.blocks if b.identity) == 5
    assert len(lw.segs) == 62
    # 4-aligned segments covering every parameter in registration order
    names = [n for n, _ in net.named_parameters()]
    assert [s.name for s in lw.segs] == names
    assert all(s.off % 4 == 0 for s in lw.segs)
    assert lw.total >= 11173962 and lw.total < 11173962 + 4 * 62
    assert lw.fc_w.param is net.linear.weight
    assert not lw.blocks[0].units[0].need_dgrad


def test_other_models_lower():
    assert lower(ResNet50(10)).blocks[1].units[2].K == 256
    lw = lower(ResNet50_ImageNet(1000))
    assert lw.blocks[0].pool == (3, 2, 1)
    lw = lower(MobileNetV2(100))
    assert sum(1 for b in lw.blocks for u in b.units if u.depthwise) == 17
    assert supports(MobileNetV2()) and supports(VGG('VGG11', 30))


@pytest.mark.parametrize('name,nconv', [('VGG11', 8), ('VGG16', 13)])
def test_vgg_lowering(name, nconv):
    """Speech VGG: one-unit blocks (conv+bias, BN, ReLU), 2x2 pools where the config has 'M',
    flatten + fc1 + fc2 head; every parameter laid out in registration order."""
    net = VGG(name, 30)
    lw = lower(net)
    assert len(lw.blocks) == nconv and lw.head_pool == 'mlp2'
    assert sum(1 for b in lw.blocks if b.pool) == 5
    assert all(b.units[0].b_seg is not None for b in lw.blocks)
    assert lw.in_channels == 1 and lw.num_classes == 30
    assert lw.fc1_w.param is net.fc1.weight and lw.fc_w.param is net.fc2.weight
    assert [s.name for s in lw.segs] == [n for n, _ in net.named_parameters()]
    assert not lw.blocks[0].need_dx and not lw.blocks[0].units[0].need_dgrad
