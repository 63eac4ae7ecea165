import numpy as np
import torch

from mercury_amd.utils import (Accuracy, Average, EMAverage, flatten, flatten_torch_tensor,
                               quantize_tensor, unflatten, unflatten_torch_tensor)
from refutil import extract, needs_ref


@needs_ref
def test_meters_match_reference():
    ns = extract('util.py', {'Average', 'EMAverage', 'Accuracy'}, {'torch': torch})
    ra, rb = ns['Average'](), Average()
    re_, rm = ns['EMAverage'](), EMAverage()
    for v, n in [(1.0, 32), (0.5, 16), (2.0, 8)]:
        ra.update(v, n)
        rb.update(v, n)
        re_.update(v)
        rm.update(v)
    assert str(ra) == str(rb)
    assert abs(re_.value - rm.value) < 1e-12 and str(re_) == str(rm)
    out = torch.randn(64, 10)
    lab = torch.randint(0, 10, (64,))
    r, m = ns['Accuracy'](), Accuracy()
    r.update(out, lab)
    m.update(out, lab)
    assert str(r) == str(m) and r.accuracy == m.accuracy


def test_average_device_lazy():
    a = Average()
    a.update(torch.tensor(2.0), 4)
    a.update(torch.tensor(4.0), 4)
    assert abs(a.average - 3.0) < 1e-6


def test_flatten_roundtrip():
    ts = [torch.randn(3, 4), [torch.randn(5), torch.randn(2, 2, 2)]]
    flat = flatten_torch_tensor(ts)
    assert flat.numel() == 12 + 5 + 8
    back = unflatten_torch_tensor(flat, ts)
    assert torch.equal(back[0], ts[0]) and torch.equal(back[1][1], ts[1][1])
    arrs = [np.arange(6).reshape(2, 3), [np.ones(4)]]
    f = flatten(arrs)
    b = unflatten(f, arrs)
    assert (b[0] == arrs[0]).all() and (b[1][0] == 1).all()


def test_quantize_unbiased():
    torch.manual_seed(0)
    a = torch.randn(2000)
    acc = torch.zeros_like(a)
    for _ in range(400):
        q = quantize_tensor(a)
        assert set(torch.unique(q.abs()).tolist()) <= {0.0, float(a.abs().max())}
        acc += q
    assert (acc / 400 - a).abs().mean() < 0.1


def test_engine_options_from_env(monkeypatch):
    """EngineOptions: defaults, and the one A/B variable (values may contain ',' and '=')."""
    from mercury_amd.config import EngineOptions
    monkeypatch.delenv('MERCURY_ENGINE_OPTS', raising=False)
    assert EngineOptions.from_env() == EngineOptions()
    monkeypatch.setenv('MERCURY_ENGINE_OPTS',
                       'hconv=score,pgemm=0,hconv_plans=32,16,128,128=64,64,1;32,8,256,256=none,'
                       'hconv_persist_grid=96')
    o = EngineOptions.from_env()
    assert o.hconv == 'score' and o.pgemm is False and o.hconv_persist_grid == 96
    assert o.hconv_plans == '32,16,128,128=64,64,1;32,8,256,256=none'
    monkeypatch.setenv('MERCURY_ENGINE_OPTS', 'no_such_option=1')
    import pytest
    with pytest.raises(ValueError):
        EngineOptions.from_env()
