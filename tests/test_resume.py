"""Checkpoint / resume semantics: a mid-epoch checkpoint resumes the partial
epoch at that epoch's LR, total step count and the per-step LR sequence equal an
uninterrupted run; per-rank resume paths; the native optimizer whitelist."""
import os
import tempfile

import pytest
import torch

from mercury_amd.ckpt import resume_path
from mercury_amd.config import Config
from mercury_amd.ops.optim import optimizer_spec
from mercury_amd.trainer import Trainer
from test_importance import FakeLoader, TinyNet


class Recording(Trainer):
    """Trainer that records (step, epoch, lr) of every step it trains."""

    def train_step(self, *a, **k):
        self.log.append((self.step, self.epoch, self.optimizer.param_groups[0]['lr']))
        return super().train_step(*a, **k)


def _make(ckdir, max_samples=10_000_000, resume=''):
    torch.manual_seed(0)
    net = TinyNet()
    cfg = Config(print_every=0, eval_every=0, log_dir=tempfile.mkdtemp(), checkpoint_dir=ckdir,
                 checkpoint_every=1, max_samples=max_samples, resume=resume, presample_batches=2)
    t = Recording(net, torch.optim.Adam(net.parameters(), lr=1e-2), FakeLoader(n=5),
                  FakeLoader(n=8), None, 'cpu', cfg)
    t.log = []
    return t


def test_mid_epoch_resume_matches_uninterrupted():
    epochs = 3
    full = _make(tempfile.mkdtemp())
    full.fit(epochs)
    assert len(full.log) == 15 and full.step == 16

    ck = tempfile.mkdtemp()
    part = _make(ck, max_samples=6)           # stops after step 6: epoch 2, 1 step done
    part.fit(epochs)
    assert [s for s, _, _ in part.log] == list(range(1, 7))
    sd = torch.load(os.path.join(ck, 'ckpt_rank0.pt'), weights_only=True)
    assert (sd['epoch'], sd['epoch_step'], sd['step']) == (2, 1, 7)

    rest = _make(tempfile.mkdtemp(), resume=ck)   # a directory resolves to ckpt_rank0.pt
    rest.fit(epochs)
    combined = part.log + rest.log
    assert [s for s, _, _ in combined] == list(range(1, 16))
    assert [e for _, e, _ in combined] == [e for _, e, _ in full.log]
    for (_, _, a), (_, _, b) in zip(combined, full.log):
        assert abs(a - b) < 1e-12
    assert rest.step == full.step


def test_resume_at_epoch_boundary():
    ck = tempfile.mkdtemp()
    part = _make(ck, max_samples=5)           # stops after the last step of epoch 1
    part.fit(2)
    rest = _make(tempfile.mkdtemp(), resume=os.path.join(ck, 'ckpt_rank{rank}.pt'))
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter('always')
        rest.fit(2)
    assert not [x for x in w if 'lr_scheduler' in str(x.message)], [str(x.message) for x in w]
    full = _make(tempfile.mkdtemp())
    full.fit(2)
    assert [(s, e) for s, e, _ in part.log + rest.log] == [(s, e) for s, e, _ in full.log]
    assert [round(l, 12) for _, _, l in part.log + rest.log] == \
        [round(l, 12) for _, _, l in full.log]
    # the first resumed step runs at epoch 2's LR, not epoch 1's again
    assert rest.log[0][1] == 2 and abs(rest.log[0][2] - full.log[5][2]) < 1e-15
    assert rest.log[0][2] != part.log[-1][2]


def test_resume_path_resolution(tmp_path):
    assert resume_path(str(tmp_path), 3) == os.path.join(str(tmp_path), 'ckpt_rank3.pt')
    assert resume_path('/x/ck_{rank}.pt', 2) == '/x/ck_2.pt'
    assert resume_path('/x/one.pt', 5) == '/x/one.pt'


def test_optimizer_whitelist():
    p = [torch.nn.Parameter(torch.zeros(4))]
    assert optimizer_spec(torch.optim.Adam(p, lr=1e-3))['algo'] == 'adam'
    s = optimizer_spec(torch.optim.AdamW(p, lr=1e-3, weight_decay=0.05))
    assert s['algo'] == 'adamw' and s['weight_decay'] == 0.05
    assert optimizer_spec(torch.optim.SGD(p, lr=0.1, momentum=0.9))['algo'] == 'sgd'
    for bad in (torch.optim.Adam(p, amsgrad=True), torch.optim.SGD(p, lr=0.1, momentum=0.9,
                                                                   nesterov=True),
                torch.optim.SGD(p, lr=0.1, momentum=0.9, dampening=0.1),
                torch.optim.SGD(p, lr=0.1), torch.optim.RMSprop(p),
                torch.optim.Adagrad(p), torch.optim.Adam(p, maximize=True),
                torch.optim.Adam([{'params': p[:1]}, {'params': [torch.nn.Parameter(
                    torch.zeros(2))]}])):
        with pytest.raises(ValueError):
            optimizer_spec(bad)
