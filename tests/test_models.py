import importlib.util
import os

import pytest
import torch

from mercury_amd.models import (MobileNetV2, MyLSTM, ResNet18, ResNet34, ResNet50,
                                ResNet50_ImageNet, ResNet101, VGG)
from refutil import REF, needs_ref


def _ref_models():
    spec = importlib.util.spec_from_file_location('ref_pytorch_model',
                                                  os.path.join(REF, 'pytorch_model.py'))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_param_counts():
    assert sum(p.numel() for p in ResNet18(10).parameters()) == 11173962
    assert sum(p.numel() for p in ResNet34(10).parameters()) == 21282122
    assert sum(p.numel() for p in ResNet50(10).parameters()) == 23520842
    assert sum(p.numel() for p in ResNet101(10).parameters()) == 42512970
    assert len(ResNet18(10).state_dict()) == 122


@needs_ref
@pytest.mark.parametrize('name', ['ResNet18', 'ResNet34', 'ResNet50'])
def test_resnet_state_dict_interchange(name):
    ref = _ref_models()
    torch.manual_seed(0)
    ours = {'ResNet18': ResNet18, 'ResNet34': ResNet34, 'ResNet50': ResNet50}[name](10)
    theirs = getattr(ref, name)(10)
    a, b = ours.state_dict(), theirs.state_dict()
    assert list(a.keys()) == list(b.keys())
    assert all(a[k].shape == b[k].shape for k in a)
    theirs.load_state_dict(a)
    ours.eval()
    theirs.eval()
    x = torch.randn(2, 3, 32, 32)
    with torch.no_grad():
        assert torch.allclose(ours(x), theirs(x), atol=1e-5)


@needs_ref
def test_vgg_interchange():
    ref = _ref_models()
    ours, theirs = VGG('VGG11', 30), ref.VGG('VGG11', 30)
    assert list(ours.state_dict()) == list(theirs.state_dict())
    theirs.load_state_dict(ours.state_dict())
    ours.eval()
    theirs.eval()
    x = torch.randn(2, 1, 101, 161)
    with torch.no_grad():
        assert torch.allclose(ours(x), theirs(x), atol=1e-5)


def test_lstm_runs_and_backprops():
    m = MyLSTM(feature_dim=40, num_classes=12, hidden_dim=32)
    x = torch.randn(4, 1, 40, 25)
    out = m(x, lengths=torch.tensor([25, 20, 10, 25]))
    assert out.shape == (4, 12)
    out.sum().backward()


def test_mobilenetv2_and_imagenet_resnet():
    m = MobileNetV2(100)
    assert m(torch.randn(2, 3, 32, 32)).shape == (2, 100)
    r = ResNet50_ImageNet(1000)
    r.eval()
    with torch.no_grad():
        assert r(torch.randn(1, 3, 224, 224)).shape == (1, 1000)
