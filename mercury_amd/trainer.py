"""The pytorch_collab train-loop API (`pytorch_collab.py:36-266`).

``Trainer(net, optimizer, train_loader, presam_loader, test_loader, device)``
with ``fit / train / evaluate / update_samples / get_next / average_model /
average_gradients`` -- same names, arguments and return shapes as the
reference.  This is the *eager* engine: it runs any ``nn.Module`` with
PyTorch ops and is the CPU path (BASELINE config 1) and the reference-
semantics oracle.  ``mercury_amd.engine.NativeTrainer`` subclasses it and
swaps the step for the MI355X kernels + HIP graphs on supported models.

Step order (reference semantics): train fwd/bwd on the batch
scored in the previous step -> score the NEXT pool with the current
(pre-update) weights -> average gradients -> optimizer step.  The batch is
one step stale and the trained images are exactly the augmented views that
were scored.

Defects fixed vs the reference: no ``torch._six``; ``next(it)``;
the global train loader is not iterated (its images were loaded and thrown
away every step) -- ``len(train_loader)`` is the step count; no per-step
``.item()`` syncs; gradients are bucketed and all-reduced while backward and
the next pool's scoring still run; initial weights (and BN buffers) are
broadcast from rank 0 unless ``parity`` asks for the reference's per-parameter
averaging; evaluation cadence is configurable and can be disabled.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch.optim.lr_scheduler import CosineAnnealingLR

from .config import Config
from .importance import pool as ispool
from .parallel.buckets import BucketedAllReduce
from .parallel.flat import FlatParams
from .utils.logging import MetricsWriter, PhaseTimer
from .utils.meters import Accuracy, Average, EMAverage


class Trainer(object):

    def __init__(self, net, optimizer, train_loader, presam_loader, test_loader, device,
                 config=None):
        self.cfg = config or Config()
        self.net = net
        self.optimizer = optimizer
        self.train_loader = train_loader
        self.presam_loader = presam_loader
        self.test_loader = test_loader
        self.device = torch.device(device)
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world_size = dist.get_world_size() if dist.is_initialized() else 1
        self.com_tensor = torch.ones(1)
        self.epoch = 0
        self.step = 1
        self.epoch_step = 0       # steps completed in the current epoch (mid-epoch resume)
        self.writer = None
        self.next_batch_iter = None
        self.computed_samples = {'index': [], 'prob': []}
        self.should_compute_importance = True
        self.batch_size = getattr(train_loader, 'batch_size', None) or self.cfg.batch_size
        self.steps_per_epoch = len(train_loader) if train_loader is not None else 1
        self.timer = PhaseTimer(self.device)
        self.scheduler = None
        self.flat = None
        self.bucketer = None
        self._setup_flat()
        self._fc_in = None
        if self.cfg.score == 'gradnorm':
            fcs = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
            if not fcs:
                raise ValueError("score='gradnorm' needs a final nn.Linear classifier")
            fcs[-1].register_forward_pre_hook(self._keep_fc_input)
        from .utils.profiling import StepWindow
        self.profile_window = StepWindow(self.cfg.profile_start, self.cfg.profile_steps)
        self.score_exchange = None
        if self.world_size > 1 and (self.cfg.global_ema or self.cfg.exchange_scores):
            from .parallel.scores import ScoreExchange
            self.score_exchange = ScoreExchange(self.cfg.pool_size(), self.device)

    def _keep_fc_input(self, _mod, inp):
        self._fc_in = inp[0].detach()

    def _score(self, output, label):
        """Per-sample importance score of a scored batch (`pytorch_collab.py:102`)."""
        if self.cfg.score == 'gradnorm':
            return ispool.classifier_gradnorm(output, label, self._fc_in)
        return F.cross_entropy(output.float(), label, reduction='none')

    # ------------------------------------------------------------------ DP plumbing
    def _setup_flat(self):
        """Move parameters into one flat buffer; attach bucketed all-reduce hooks."""
        self.flat = FlatParams(self.net)
        if self.world_size == 1:
            return
        bb = int(self.cfg.bucket_mb * (1 << 20)) or None
        self.bucketer = BucketedAllReduce(self.flat, bb, average=True,
                                          wire_dtype=torch.bfloat16 if self.cfg.wire_bf16 else None)
        if self.cfg.overlap and not self.cfg.parity:
            self.bucketer.attach()

    def average_model(self):
        """Initial replica sync (`pytorch_collab.py:84-87`)."""
        if self.world_size == 1:
            return
        if self.cfg.parity:
            # reference: one all-reduce(SUM)/W per parameter tensor, buffers not synced
            for p in self.net.parameters():
                dist.all_reduce(p.data, op=dist.ReduceOp.SUM)
                p.data /= float(self.world_size)
            return
        with torch.no_grad():
            dist.broadcast(self.flat.data, 0)
            for b in self.net.buffers():
                dist.broadcast(b, 0)

    def average_gradients(self):
        """Gradient average (`pytorch_collab.py:236-249`) on the flat buffer."""
        if self.world_size == 1:
            return
        self.flat.relink_grads()
        if self.bucketer is not None and self.bucketer._hooks:
            self.bucketer.finish()
        else:
            self.bucketer.allreduce_now()

    # ------------------------------------------------------------------ sampling
    def get_next(self):
        if self.next_batch_iter is None:
            self.next_batch_iter = iter(self.presam_loader)
        try:
            return next(self.next_batch_iter)
        except StopIteration:
            self.next_batch_iter = iter(self.presam_loader)
            return next(self.next_batch_iter)

    def update_samples(self, ema_loss, alpha=None):
        """Score a presample pool and draw the next training batch (`pytorch_collab.py:89-117`).

        Returns ``(weights = N*p[idx], data[idx], label[idx], index[idx], pool_mean)``."""
        alpha = self.cfg.alpha if alpha is None else alpha
        if not self.cfg.importance and self.score_exchange is None:
            # uniform-sampling baseline (the native engine's too): the next loader batch with
            # unit weights -- no presample pool is scored
            idx, data, label = self.get_next()
            data = data.to(self.device, non_blocking=True)
            label = torch.as_tensor(label).to(self.device, non_blocking=True)
            return (torch.ones(data.shape[0], device=self.device), data, label,
                    torch.as_tensor(idx), torch.zeros((), device=self.device))
        losses, labels, datas, index = [], [], [], []
        cnt = 0
        with torch.no_grad():
            while self.should_compute_importance and cnt < self.cfg.presample_batches:
                cnt += 1
                idx, data, label = self.get_next()
                data = data.to(self.device, non_blocking=True)
                label = torch.as_tensor(label).to(self.device, non_blocking=True)
                output = self.net(data)  # train mode: BN batch stats, as the reference
                losses.append(self._score(output, label))
                labels.append(label)
                datas.append(data)
                index.append(torch.as_tensor(idx))
                if not self._global_ema():
                    # EMA updated with the running pool mean after each batch
                    ema_loss.update(torch.cat(losses).mean())
        pool_losses = torch.cat(losses)
        pool_mean = pool_losses.mean()
        if self.score_exchange is not None and cnt == self.cfg.presample_batches:
            self.score_exchange.start(pool_losses.float())
            if self._global_ema():
                # one normaliser for every rank: the replay runs over the global pool means
                g = self.score_exchange.wait()
                ispool.ema_replay(ema_loss, ispool.global_cumulative_means(g, self.batch_size))
                pool_mean = g.mean()
        if self.cfg.importance:
            probs = ispool.importance_probs(pool_losses, ema_loss.value, alpha)
        else:
            probs = torch.full_like(pool_losses, 1.0 / pool_losses.numel())
        important_idx = ispool.draw(probs, self.batch_size)
        weights = ispool.is_weights(probs, important_idx)
        return (weights, torch.cat(datas)[important_idx], torch.cat(labels)[important_idx],
                torch.cat(index)[important_idx.cpu()], pool_mean)

    def _global_ema(self):
        return self.cfg.global_ema and self.score_exchange is not None

    # ------------------------------------------------------------------ loop
    def train_step(self, probs, i_data, i_label, ema, running_loss, running_acc):
        t = self.timer.start('fwd_bwd')
        output = self.net(i_data)
        losses = F.cross_entropy(output.float(), i_label, reduction='none')
        running_acc.update(output, i_label)
        loss = ispool.weighted_loss(losses, probs)
        self.flat.zero_grad()
        loss.backward()
        self.timer.stop(t)
        t = self.timer.start('score')
        self.should_compute_importance = True
        nxt = self.update_samples(ema)
        self.timer.stop(t)
        t = self.timer.start('sync')
        self.average_gradients()
        self.timer.stop(t)
        t = self.timer.start('opt')
        self.optimizer.step()
        self.timer.stop(t)
        running_loss.update(loss.detach(), self.batch_size)
        return nxt, loss

    def train(self):
        running_train_loss = Average()
        presam_ema_loss = EMAverage(self.cfg.ema_alpha)
        runing_train_acc = Accuracy()
        probs, i_data, i_label, _, _ = self.update_samples(presam_ema_loss)
        for _ in range(max(0, self.steps_per_epoch - self.epoch_step)):
            t0 = time.perf_counter()
            (probs, i_data, i_label, _, _), _ = self.train_step(
                probs, i_data, i_label, presam_ema_loss, running_train_loss, runing_train_acc)
            self._after_step(running_train_loss, runing_train_acc, presam_ema_loss, t0)
            self._advance()
            if self._stop():
                break
        return running_train_loss, runing_train_acc, presam_ema_loss

    def _advance(self):
        """Count a finished step, then checkpoint on cadence.  Restored exactly on resume: the
        step counter ("``epoch_step`` steps of epoch ``epoch`` done, ``step`` is the next
        step"), so the resumed run finishes the partial epoch before the LR scheduler advances
        and follows the same LR sequence (see ``fit``), plus weights and optimizer state.  NOT
        restored by the eager Trainer: the presample-iterator position and the pending scored
        pool -- a mid-epoch resume re-primes ``update_samples`` from a fresh iterator, so the
        data order (and hence the losses) after the resume differ from an uninterrupted run.
        (The native engine's checkpoint also carries its counters, EMA and importance table.)"""
        self.step += 1
        self.epoch_step += 1
        cfg = self.cfg
        if cfg.checkpoint_dir and cfg.checkpoint_every and \
                (self.step - 1) % cfg.checkpoint_every == 0:
            from .ckpt import save_checkpoint
            save_checkpoint(self, os.path.join(cfg.checkpoint_dir, 'ckpt_rank%d.pt' % self.rank))

    def _stop(self):
        return self.step * self.world_size > self.cfg.max_samples

    def _flat_params(self):
        return self.flat.data

    def _health(self):
        """Replica-divergence check + profiler window, once per step."""
        cfg = self.cfg
        self.profile_window.step(self.step)
        if cfg.check_replicas_every and self.world_size > 1 and \
                self.step % cfg.check_replicas_every == 0:
            from .parallel.health import ReplicaDivergence, check_replicas
            ok, spread = check_replicas(self._flat_params(), rtol=cfg.replica_rtol)
            if not ok:
                msg = 'rank %d: DP replicas diverged at step %d (relative spread %.3g)' % (
                    self.rank, self.step, spread)
                if cfg.on_divergence == 'raise':
                    raise ReplicaDivergence(msg)
                print('[mercury_amd] WARNING ' + msg, flush=True)

    def _after_step(self, running_loss, running_acc, ema, t0):
        cfg = self.cfg
        self._health()
        if cfg.print_every and self.step % cfg.print_every == 0 and self.rank == 0:
            ph = self.timer.collect()
            print('step:{}, running train loss: {}, running train acc: {}, presam_ema_loss: {}, '
                  'step time:{:.3f}, {}'.format(
                      self.step, running_loss, running_acc, ema, time.perf_counter() - t0,
                      ', '.join('{}:{:.3f}ms'.format(k, v) for k, v in ph.items())), flush=True)
        if cfg.eval_every and self.step % cfg.eval_every == 0 and (
                self.rank == 0 or cfg.eval_all_ranks):
            train_loss, train_acc, test_loss, test_acc = self.evaluate()
            if self.writer is not None:
                self.writer.add_scalar('train/acc', train_acc.accuracy, self.step)
                self.writer.add_scalar('test/acc', test_acc.accuracy, self.step)
                self.writer.add_scalar('train/loss', train_loss.average, self.step)
                self.writer.add_scalar('test/loss', test_loss.average, self.step)
            if self.rank == 0:
                print('(Eval) Step: {}, train loss: {}, train acc: {} test loss: {}, test acc: {}'
                      .format(self.step, train_loss, train_acc, test_loss, test_acc), flush=True)

    def fit(self, epochs):
        if self.rank == 0:
            self.writer = MetricsWriter(self.cfg.log_dir or self.cfg.default_log_dir(
                self.world_size))
        self.scheduler = CosineAnnealingLR(self.optimizer, epochs)
        if self.cfg.resume:
            from .ckpt import load_checkpoint, resume_path
            load_checkpoint(self, resume_path(self.cfg.resume, self.rank))
        self.average_model()
        stopped = False
        if self.epoch_step > 0:
            # resumed inside epoch ``self.epoch``: finish it at that epoch's LR, then advance
            if self.epoch_step < self.steps_per_epoch:
                self.train()
            stopped = self._stop()
            if self.epoch_step >= self.steps_per_epoch:
                # resumed exactly at an epoch's end: this process has not stepped the optimizer
                # yet, but the checkpointed run did -- advancing the restored schedule here
                # reproduces the uninterrupted run's LR sequence (tests/test_resume.py), so
                # torch's "scheduler before optimizer" warning does not apply
                import warnings
                with warnings.catch_warnings():
                    warnings.filterwarnings('ignore', message='Detected call of `lr_scheduler')
                    self.scheduler.step()
        for epoch in range(self.epoch + 1, epochs + 1):
            if stopped:
                break
            self.epoch = epoch
            self.epoch_step = 0
            self.train()
            if self.epoch_step >= self.steps_per_epoch:
                self.scheduler.step()
            stopped = self._stop()
        self.profile_window.close()
        if self.writer is not None:
            self.writer.close()

    def evaluate(self, max_batches=None):
        test_loss, test_acc = Average(), Accuracy()
        train_loss, train_acc = Average(), Accuracy()
        self.net.eval()
        with torch.no_grad():
            for loader, lm, am in ((self.train_loader, train_loss, train_acc),
                                   (self.test_loader, test_loss, test_acc)):
                if loader is None:
                    continue
                for i, (_, data, label) in enumerate(loader):
                    if max_batches is not None and i >= max_batches:
                        break
                    data = data.to(self.device)
                    label = torch.as_tensor(label).to(self.device)
                    output = self.net(data)
                    lm.update(F.cross_entropy(output.float(), label), data.size(0))
                    am.update(output, label)
        self.net.train()
        return train_loss, train_acc, test_loss, test_acc

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self):
        return {'model': self.net.state_dict(),
                'optimizer': self.optimizer.state_dict(),
                'scheduler': self.scheduler.state_dict() if self.scheduler else None,
                'step': self.step, 'epoch': self.epoch, 'epoch_step': self.epoch_step}

    def load_state_dict(self, sd):
        self.net.load_state_dict(sd['model'])
        self.optimizer.load_state_dict(sd['optimizer'])
        if sd.get('scheduler') and self.scheduler is not None:
            self.scheduler.load_state_dict(sd['scheduler'])
        self.step = sd['step']
        self.epoch = sd['epoch']
        self.epoch_step = int(sd.get('epoch_step', 0))
