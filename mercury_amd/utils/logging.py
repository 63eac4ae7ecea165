"""Metrics writers and phase timers.

``MetricsWriter`` has tensorboardX's ``add_scalar(tag, value, step)`` surface
(the reference writes ``train/acc``, ``test/acc``, ``train/loss``,
``test/loss``, `pytorch_collab.py:187-190`) and appends JSON lines to
``<log_dir>/metrics.jsonl``; if tensorboardX happens to be importable it
mirrors to it.  ``PhaseTimer`` brackets phases with HIP events on the GPU
(``time.time()`` deltas in the reference are async-skewed) and is
read back only at log cadence.
"""
from __future__ import annotations

import json
import os
import time

import torch


class MetricsWriter(object):

    def __init__(self, log_dir):
        self.log_dir = log_dir
        os.makedirs(log_dir, exist_ok=True)
        self._f = open(os.path.join(log_dir, 'metrics.jsonl'), 'a')
        self._tb = None
        try:  # optional
            from tensorboardX import SummaryWriter  # noqa: F401
            self._tb = SummaryWriter(log_dir)
        except Exception:
            self._tb = None

    def add_scalar(self, tag, value, step):
        if torch.is_tensor(value):
            value = float(value.item())
        self._f.write(json.dumps({'tag': tag, 'value': float(value), 'step': int(step),
                                  'time': time.time()}) + '\n')
        self._f.flush()
        if self._tb is not None:
            self._tb.add_scalar(tag, value, step)

    def close(self):
        self._f.close()
        if self._tb is not None:
            self._tb.close()


class PhaseTimer(object):
    """Accumulates per-phase device time with event pairs (no per-step sync)."""

    def __init__(self, device):
        self.cuda = torch.device(device).type == 'cuda'
        self.pending = []
        self.totals = {}
        self.counts = {}

    def start(self, name):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return (name, e)
        return (name, time.perf_counter())

    def stop(self, tok):
        name, s = tok
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.pending.append((name, s, e))
        else:
            self._add(name, (time.perf_counter() - s) * 1e3)

    def _add(self, name, ms):
        self.totals[name] = self.totals.get(name, 0.0) + ms
        self.counts[name] = self.counts.get(name, 0) + 1

    def collect(self):
        if self.pending:
            self.pending[-1][2].synchronize()
            for name, s, e in self.pending:
                self._add(name, s.elapsed_time(e))
            self.pending = []
        out = {k: self.totals[k] / max(self.counts[k], 1) for k in self.totals}
        self.totals, self.counts = {}, {}
        return out
