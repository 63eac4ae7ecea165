"""Multi-process CPU tests over gloo (SURVEY §4 layer 3)."""
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from mercury_amd.parallel import (BucketedAllReduce, FlatParams, ScoreExchange, allreduce,
                                  spawn)


def _ring(rank, ws, numel):
    torch.manual_seed(rank)
    t = torch.randn(numel)
    out = allreduce(t)
    ref = t.clone()
    dist.all_reduce(ref)
    assert torch.allclose(out, ref, atol=1e-5), (rank, numel)
    avg = allreduce(t, op='avg')
    assert torch.allclose(avg, ref / ws, atol=1e-5)


@pytest.mark.parametrize('ws', [2, 3, 4])
def test_ring_allreduce(ws):
    for numel in (1, ws - 1, 1000, 1001):
        if numel >= 1:
            spawn(_ring, ws, args=(numel,))


class Small(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(16, 64)
        self.b = nn.Linear(64, 64)
        self.c = nn.Linear(64, 10)

    def forward(self, x):
        return self.c(F.relu(self.b(F.relu(self.a(x)))))


def _bucketed(rank, ws):
    torch.manual_seed(0)
    m = Small()
    flat = FlatParams(m)
    torch.manual_seed(100 + rank)
    x = torch.randn(8, 16)
    # local gradient first, without hooks: once attached, a bucket's async all-reduce may
    # already be rewriting flat.grad in place while backward is still running
    flat.zero_grad()
    m(x).pow(2).mean().backward()
    local = flat.grad.clone()
    br = BucketedAllReduce(flat, bucket_bytes=4096).attach()
    assert len(br.buckets) > 1
    flat.zero_grad()
    m(x).pow(2).mean().backward()
    br.finish()
    ref = local.clone()
    dist.all_reduce(ref)
    assert torch.allclose(flat.grad, ref / ws, atol=1e-6)
    # score exchange
    se = ScoreExchange(5, 'cpu').start(torch.full((5,), float(rank)))
    g = se.wait()
    assert torch.equal(g[:, 0], torch.arange(ws, dtype=torch.float32))


def test_bucketed_allreduce_overlap_hooks():
    spawn(_bucketed, 2)


def _trainer_dp(rank, ws):
    from mercury_amd.config import Config
    from mercury_amd.trainer import Trainer
    from test_importance import FakeLoader, TinyNet
    torch.manual_seed(rank)            # different init per rank: broadcast must fix it
    net = TinyNet()
    cfg = Config(print_every=0, eval_every=0, bucket_mb=0.001, log_dir=tempfile.mkdtemp())
    opt = torch.optim.Adam(net.parameters(), lr=1e-3)
    loader = FakeLoader(n=6, seed=rank)   # non-IID: different shards
    t = Trainer(net, opt, FakeLoader(n=4), loader, None, 'cpu', cfg)
    t.fit(2)
    flat = t.flat.data.clone()
    gathered = [torch.zeros_like(flat) for _ in range(ws)]
    dist.all_gather(gathered, flat)
    for g in gathered:
        assert torch.equal(g, gathered[0]), 'replicas diverged'
    assert t.step == 9


def test_trainer_dp_replicas_identical():
    spawn(_trainer_dp, 2)


def _global_ema(rank, ws):
    from mercury_amd.config import Config
    from mercury_amd.trainer import Trainer
    from mercury_amd.utils import EMAverage
    from test_importance import FakeLoader, TinyNet
    torch.manual_seed(0)
    net = TinyNet()
    cfg = Config(print_every=0, eval_every=0, global_ema=True, score='gradnorm',
                 log_dir=tempfile.mkdtemp())
    t = Trainer(net, torch.optim.Adam(net.parameters(), lr=1e-3), FakeLoader(n=4),
                FakeLoader(n=12, seed=rank), None, 'cpu', cfg)
    ema = EMAverage()
    w, d, lab, idx, pm = t.update_samples(ema)
    assert w.shape == (32,) and torch.isfinite(w).all()
    vals = [torch.zeros(1) for _ in range(ws)]
    dist.all_gather(vals, torch.tensor([float(ema.value)]))
    assert vals[0].item() == vals[1].item(), 'global EMA must agree across ranks'
    g = t.score_exchange.wait()
    assert g.shape == (ws, 320) and abs(float(pm) - float(g.mean())) < 1e-6


def test_trainer_global_ema_gradnorm_two_ranks():
    spawn(_global_ema, 2)


def _health(rank, ws):
    from mercury_amd.parallel.health import check_replicas, replica_fingerprint
    from mercury_amd.config import Config
    from mercury_amd.trainer import Trainer
    from test_importance import FakeLoader, TinyNet
    flat = torch.arange(1000, dtype=torch.float32) / 7
    ok, spread = check_replicas(flat)
    assert ok and spread == 0.0
    bad = flat.clone()
    if rank == 1:
        bad[3], bad[4] = bad[4].item(), bad[3].item()    # a permutation: same sum / sumsq
    ok, spread = check_replicas(bad)
    assert not ok and spread > 0
    assert replica_fingerprint(flat).shape == (3,)
    # the trainer checks every step and keeps training (replicas stay identical)
    torch.manual_seed(rank)
    net = TinyNet()
    cfg = Config(print_every=0, eval_every=0, check_replicas_every=1,
                 log_dir=tempfile.mkdtemp())
    t = Trainer(net, torch.optim.Adam(net.parameters(), lr=1e-3), FakeLoader(n=3),
                FakeLoader(n=6, seed=rank), None, 'cpu', cfg)
    t.fit(1)


def test_replica_divergence_check():
    spawn(_health, 2)
