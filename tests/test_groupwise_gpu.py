"""Native global-table sampling mode (engine ``sampler='groupwise'``) on a real GPU.

Reference semantics (``Groupwise_Sampler``, `util.py:94-160`): every iteration scores the next
contiguous slice of the dataset into the global importance table under a NEW group id, and the
training batch is drawn from the current group with ``p ~ imp + mean(imp)``.  Natively the
table lives in HBM (csrc/table.hip), the slice is scored by the engine's B=320 forward, and the
draw + pool-slot mapping + importance weights are three graph-captured launches.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    x, y = synthetic_arrays(2000, 10, seed=5)
    torch.manual_seed(7)
    net = ResNet18(10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, seed=3, sampler='groupwise', **kw)
    eng.set_shard(x, y)
    return eng


def _check_batch(eng):
    """The drawn batch comes from the current group = the slice scored last, with weights
    n_group * (imp + mean) / total."""
    sm, tab = eng.score_mode, eng.table
    torch.cuda.synchronize()
    stamp = int(eng._gstamp.item())
    pos = sm.index.long()
    Ns = eng.shard.shape[0]
    start = int(pos[0])
    assert torch.equal(pos.cpu(), (torch.arange(eng.P) + start) % Ns)   # contiguous slice
    members = torch.nonzero(tab.group == stamp).flatten()
    assert torch.equal(members.sort().values.cpu(), pos.sort().values.cpu())
    idx = eng.idx.long()
    assert int(idx.min()) >= 0 and int(idx.max()) < eng.P
    drawn = pos[idx]
    assert bool((tab.group[drawn] == stamp).all())
    imp = tab.importance[members].double()
    mean = imp.mean()
    total = (imp + mean).sum()
    want = (len(members) * (tab.importance[drawn].double() + mean) / total).float()
    assert torch.allclose(eng.isw, want, rtol=1e-4, atol=1e-6)
    # the pool's losses were scattered into the table for exactly these positions
    assert torch.allclose(tab.importance[pos], sm.losses)


def test_groupwise_engine_steps_eager_and_graphs():
    eng = _engine()
    eng.prime()
    _check_batch(eng)
    s0 = int(eng._gstamp.item())
    eng.step()
    _check_batch(eng)
    eng.build_graphs()
    for _ in range(4):
        eng.step()
    _check_batch(eng)
    torch.cuda.synchronize()
    assert int(eng._gstamp.item()) == s0 + 5          # a new group per scored slice
    m = eng.read_meters()
    assert np.isfinite(m['loss_sum']) and m['count'] == 32 * 5
    assert np.isfinite(m['pool_mean']) and m['pool_mean'] > 0


@pytest.mark.parametrize('N', [50000, 1281167])
def test_groupwise_draws_match_cpu_sampler_chi2(N):
    """Draw distribution of the HBM table (draw_batch) vs the CPU Groupwise_Sampler's
    normalised group weights, chi-square over the group's members."""
    from mercury_amd.importance.groupwise import Groupwise_Sampler
    from mercury_amd.ops.table import ImportanceTable

    class DS:
        def __len__(self):
            return N
    P = 320
    g = torch.Generator().manual_seed(N)
    start = int(torch.randint(0, N - P, (1,), generator=g))
    losses = torch.rand(P, generator=g) * 3.0
    # CPU oracle: same table content (group 1 = [start, start + P))
    cpu = Groupwise_Sampler(DS())
    cpu.cur_sample_index = start
    cpu.update_importance(1, P, None, losses=losses)
    members, p = cpu.group_distribution()
    tab = ImportanceTable(N, 'cuda')
    pool_index = torch.arange(start, start + P, dtype=torch.int32, device='cuda')
    stamp = torch.ones(1, dtype=torch.int64, device='cuda')
    tab.scatter(pool_index, losses.cuda(), stamp=stamp)
    nd = 200_000
    pos32 = torch.empty(nd, dtype=torch.int32, device='cuda')
    idx = torch.empty(nd, dtype=torch.int32, device='cuda')
    isw = torch.empty(nd, dtype=torch.float32, device='cuda')
    tab.draw_batch(nd, stamp, pos32, pool_index, N, P, idx, isw, seed=11)
    torch.cuda.synchronize()
    assert torch.equal(pos32.long(), idx.long() + start)
    counts = torch.bincount(idx.long().cpu(), minlength=P).double()
    exp = p.double() * nd
    assert torch.equal(members.cpu(), torch.arange(start, start + P))
    chi2 = float(((counts - exp) ** 2 / exp).sum())
    dof = P - 1
    assert chi2 < dof + 6 * (2 * dof) ** 0.5, chi2
    # weights n_group * p of each draw
    assert torch.allclose(isw.cpu().double(), (P * p.double())[idx.long().cpu()], rtol=1e-4)


def test_groupwise_trainer_checkpoint_roundtrip(tmp_path):
    import os
    from mercury_amd.ckpt import load_checkpoint, save_checkpoint
    from mercury_amd.collab import make_trainer
    from mercury_amd.config import Config
    from mercury_amd.data import load_cifar10_noniid
    from mercury_amd.models import ResNet18
    np.random.seed(102)
    pres, train, test = load_cifar10_noniid(1, 0.5, data_dir='/nonexistent')
    cfg = Config(num_epochs=1, max_samples=20, print_every=10, eval_every=0,
                 log_dir=str(tmp_path), sampler='groupwise')
    torch.manual_seed(0)
    net = ResNet18(10).cuda()
    tr = make_trainer(cfg, net, torch.optim.Adam(net.parameters(), lr=1e-3), train, pres[0],
                      test, 'cuda')
    tr.fit(1)
    assert tr.engine.sampler == 'groupwise' and int((tr.engine.table.group > 0).sum()) > 0
    path = save_checkpoint(tr, os.path.join(tmp_path, 'ck.pt'))
    torch.manual_seed(1)
    net2 = ResNet18(10).cuda()
    tr2 = make_trainer(cfg, net2, torch.optim.Adam(net2.parameters(), lr=1e-3), train, pres[0],
                       test, 'cuda')
    load_checkpoint(tr2, path)
    assert torch.equal(tr2.engine.table.importance, tr.engine.table.importance)
    assert torch.equal(tr2.engine.table.group, tr.engine.table.group)
    assert torch.equal(tr2.engine.ctrl, tr.engine.ctrl)
