"""Per-phase DEVICE timing of the native step (reference C27: `pytorch_collab.py:129-178`
prints step / ff / bp / sync / IS times).

The native step is a handful of asynchronous graph replays on three streams, so host
timestamps (or roctx ranges around the replays) time the host issue, not the work.  Here
each phase boundary is a HIP event recorded on the stream that runs the phase:

    step   : start of the step on the train stream  -> end of its tail
    score  : scoring-stream start -> end (pool build, B=320 forward, scores, draw)
    train  : train-stream forward + backward (all bucket segments)
    comm   : sum over buckets of the all-reduce's own span on the comm stream
    wait   : end of backward -> start of the tail (the train stream waiting for the scoring
             stream and the last all-reduce: the exposed part of both)
    tail   : BN running stats + optimizer + weight copies + next-batch gather
    comm_exposed : last all-reduce end - end of backward (> 0: communication on the
             critical path)
    score_xchg : the cross-worker score all-gather on the score stream (0 when off)

``critical = max(score, train + wait) + tail`` reproduces ``step`` (the check printed by
``NativeTrainer`` at ``print_every``).  Events are pre-allocated; recording costs a few
microseconds of host time per event, so timing is enabled only for the steps that are read.
"""
from __future__ import annotations

import torch


class StepTimer(object):

    def __init__(self, device, max_buckets=64):
        self.device = device
        self.on = False
        self._ev = {}
        self._nb = 0
        self.max_buckets = max_buckets
        self._pending = False

    def _event(self, key):
        ev = self._ev.get(key)
        if ev is None:
            ev = self._ev[key] = torch.cuda.Event(enable_timing=True)
        return ev

    def mark(self, key, stream):
        if self.on:
            self._event(key).record(stream)
            self._pending = True

    def bucket(self, i, end, stream):
        if self.on and i < self.max_buckets:
            self._event(('b', i, end)).record(stream)
            self._nb = max(self._nb, i + 1)

    def begin_step(self):
        self._nb = 0

    def collect(self):
        """Milliseconds per phase of the last timed step (synchronises on its last event)."""
        if not self._pending:
            return {}
        ev = self._ev
        ev['end'].synchronize()

        def d(a, b):
            return ev[a].elapsed_time(ev[b]) if a in ev and b in ev else 0.0
        out = {'step': d('start', 'end'), 'score': d('score0', 'score1'),
               'train': d('start', 'train1'), 'wait': d('train1', 'tail0'),
               'tail': d('tail0', 'end')}
        comm = [ev[('b', i, 0)].elapsed_time(ev[('b', i, 1)]) for i in range(self._nb)]
        out['comm'] = sum(comm)
        # the score all-gather's span on the score stream (DP with exchange_scores / global_ema)
        out['score_xchg'] = d('xchg0', 'xchg1')
        out['comm_buckets'] = comm
        if self._nb:
            out['comm_exposed'] = max(0.0, d('train1', ('b', self._nb - 1, 1)))
            # fraction of all-reduce time hidden under the backward / scoring work
            out['overlap'] = 1.0 - min(out['comm_exposed'], out['comm']) / max(out['comm'], 1e-9)
        out['critical'] = max(out['score'], out['train'] + out['wait']) + out['tail']
        self._pending = False
        return out
