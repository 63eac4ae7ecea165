import numpy as np
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from mercury_amd.config import Config
from mercury_amd.importance import (Groupwise_Sampler, alias_distribution, alias_draw,
                                    build_alias, cumulative_means, ema_replay, importance_probs)
from mercury_amd.trainer import Trainer
from mercury_amd.utils import EMAverage
from refutil import extract, extract_method, needs_ref


class TinyNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.conv = nn.Conv2d(3, 4, 3, padding=1)
        self.bn = nn.BatchNorm2d(4)
        self.fc = nn.Linear(4, 10)

    def forward(self, x):
        return self.fc(F.relu(self.bn(self.conv(x))).mean((2, 3)))


class FakeLoader:
    def __init__(self, n=20, b=32, seed=0):
        g = torch.Generator().manual_seed(seed)
        self.batches = [(torch.arange(i * b, (i + 1) * b), torch.randn(b, 3, 8, 8, generator=g),
                         torch.randint(0, 10, (b,), generator=g)) for i in range(n)]
        self.batch_size = b

    def __iter__(self):
        return iter(self.batches)

    def __len__(self):
        return len(self.batches)


@needs_ref
def test_update_samples_matches_reference(monkeypatch):
    torch.manual_seed(0)
    net = TinyNet()
    loader = FakeLoader()
    ns = {'torch': torch, 'F': F}
    exec(extract_method('pytorch_collab.py', 'Trainer', 'update_samples').replace(
        'def update_samples', 'def ref_update_samples', 1).replace('\n    ', '\n'), ns)
    refm = extract('util.py', {'EMAverage'}, {'torch': torch})

    class FakeSelf:
        pass
    fs = FakeSelf()
    fs.net, fs.device, fs.train_loader = net, 'cpu', loader
    fs.should_compute_importance = True
    fs.it = iter(loader)
    fs.get_next = lambda: next(fs.it)
    # deterministic stand-in for multinomial so both sides draw the same indices
    monkeypatch.setattr(torch, 'multinomial',
                        lambda p, k, replacement=True, generator=None:
                        torch.argsort(p, descending=True)[:k].repeat(1))
    ema_r = refm['EMAverage']()
    bn_state = {k: v.clone() for k, v in net.state_dict().items()}
    r = ns['ref_update_samples'](fs, ema_r, 0.5)

    net.load_state_dict(bn_state)
    t = Trainer(net, torch.optim.Adam(net.parameters()), loader, loader, None, 'cpu', Config())
    t.next_batch_iter = iter(loader)
    ema_m = EMAverage()
    m = t.update_samples(ema_m, 0.5)
    assert abs(float(ema_r.value) - float(ema_m.value)) < 1e-6
    for a, b in zip(r, m):
        assert torch.allclose(torch.as_tensor(a).float(), torch.as_tensor(b).float(), atol=1e-5)
    # BN running stats mutated by scoring in train mode, 10 updates
    assert int(net.bn.num_batches_tracked) == 10


def test_ema_replay_equals_incremental():
    torch.manual_seed(1)
    losses = torch.rand(320) * 3
    inc = EMAverage()
    for j in range(10):
        inc.update(losses[:32 * (j + 1)].mean())
    rep = ema_replay(EMAverage(), cumulative_means(losses, 32))
    assert abs(float(inc.value) - float(rep.value)) < 1e-6


def test_is_estimator_unbiased():
    # E_j~p[l_j / (N p_j)] = mean(l)
    torch.manual_seed(0)
    losses = torch.rand(320) * 2
    p = importance_probs(losses, 0.4, 0.5)
    idx = torch.multinomial(p, 200000, replacement=True)
    est = (losses[idx] / (p[idx] * 320)).mean()
    assert abs(float(est) - float(losses.mean())) < 0.01


def test_alias_table_exact_and_statistical():
    rng = np.random.RandomState(0)
    p = rng.rand(320) ** 3
    p /= p.sum()
    prob, alias = build_alias(p)
    assert np.allclose(alias_distribution(prob, alias), p, atol=1e-12)
    draws = alias_draw(prob, alias, rng.rand(400000), rng.rand(400000))
    freq = np.bincount(draws, minlength=320) / 400000
    chi2 = ((freq - p) ** 2 / p).sum() * 400000
    assert chi2 < 320 + 6 * np.sqrt(2 * 320)


class SliceDS:
    def __init__(self, n=100):
        self.x = torch.randn(n, 3, 8, 8)
        self.y = torch.randint(0, 10, (n,))

    def __len__(self):
        return len(self.x)

    def get_slice(self, s, e):
        return self.x[s:e], self.y[s:e]


@needs_ref
def test_groupwise_lifecycle_matches_reference():
    ns = extract('util.py', {'Groupwise_Sampler'},
                 {'np': np, 'torch': torch, 'F': F, 'Sampler': object})
    ds = SliceDS(100)
    net = TinyNet()
    net.eval()
    ref = ns['Groupwise_Sampler'](ds)
    ours = Groupwise_Sampler(ds)
    for it, bs in [(0, 30), (0, 30), (1, 50), (2, 40), (2, 40)]:
        with torch.no_grad():
            ref.update_importance(it, bs, net, device='cpu')
        ours.update_importance(it, bs, net, device='cpu')
        assert ref.group_index == ours.group_index
        assert ref.cur_sample_index == ours.cur_sample_index
        assert np.array_equal(ref.group_indicator, ours.group_indicator.numpy().astype(float))
        assert np.allclose(ref.importance, ours.importance.numpy(), atol=1e-5)
    members, p = ours.group_distribution()
    draws = [i for _, i in zip(range(200), iter(ours))]
    assert set(draws) <= set(members.tolist())
    assert len(ours) == 100
    assert len(list(iter(Groupwise_Sampler(ds)))) == 100  # stops after len(dataset) yields


def test_global_cumulative_means_and_gradnorm():
    from mercury_amd.importance.pool import (classifier_gradnorm, cumulative_means,
                                             global_cumulative_means)
    torch.manual_seed(0)
    x = torch.rand(320)
    assert torch.allclose(global_cumulative_means(x[None], 32), cumulative_means(x, 32))
    g = torch.rand(3, 320)
    gm = global_cumulative_means(g, 32)
    assert torch.allclose(gm[4], g[:, :160].mean())
    # gradnorm == per-sample autograd norm of the classifier's (W, b) gradient
    fc = nn.Linear(20, 7)
    h = torch.randn(5, 20)
    y = torch.randint(0, 7, (5,))
    gn = classifier_gradnorm(fc(h), y, h)
    for i in range(5):
        fc.zero_grad()
        F.cross_entropy(fc(h[i:i + 1]), y[i:i + 1]).backward()
        ref = torch.sqrt(fc.weight.grad.pow(2).sum() + fc.bias.grad.pow(2).sum())
        assert torch.allclose(gn[i], ref, atol=1e-5)
