"""Metric meters.

Host meters keep the reference field names and string formats
(`util.py:183-238`: ``Average``, ``EMAverage``, ``Accuracy``).  The reference
syncs the device on every ``update`` (``.item()`` in ``Accuracy.update``,
``util.py:228``); here ``Accuracy`` and ``Average`` accept device tensors and
keep them on device until someone reads ``.accuracy`` / ``.average`` -- the
hot loop never forces a device->host sync.  The native engine's graph-captured
form is its fixed ``meters`` buffer (engine/native.py): kernels accumulate into
it and it is read back only at log cadence (``read_meters``).
"""
from __future__ import annotations

import torch


def _to_float(v):
    if torch.is_tensor(v):
        return float(v.detach().float().item())
    return float(v)


class Average(object):
    """Weighted running mean (`util.py:183-199`)."""

    def __init__(self):
        self.sum = 0
        self.count = 0

    def update(self, value, number):
        # value may be a device scalar: accumulate lazily, no sync here.
        if torch.is_tensor(value):
            value = value.detach()
        self.sum = self.sum + value * number
        self.count += number

    @property
    def average(self):
        return _to_float(self.sum) / self.count

    def __str__(self):
        return '{:.6f}'.format(self.average)


class EMAverage(object):
    """Exponential moving average, first update sets the value (`util.py:200-214`)."""

    def __init__(self, alpha=0.9):
        self.first_update = True
        self.value = 0
        self.alpha = alpha

    def update(self, value):
        if self.first_update:
            self.value = value
            self.first_update = False
        else:
            self.value = self.alpha * self.value + (1 - self.alpha) * value

    def state_dict(self):
        v = self.value
        return {'first_update': self.first_update,
                'value': _to_float(v) if torch.is_tensor(v) or isinstance(v, float) else v,
                'alpha': self.alpha}

    def load_state_dict(self, sd):
        self.first_update = sd['first_update']
        self.value = sd['value']
        self.alpha = sd['alpha']

    def __str__(self):
        return '{:.6f}'.format(_to_float(self.value))


class Accuracy(object):
    """Top-1 accuracy (`util.py:216-238`), device-resident correct count."""

    def __init__(self):
        self.correct = 0
        self.count = 0

    def update(self, output, label):
        predictions = output.detach().argmax(dim=1)
        correct = predictions.eq(label.detach()).sum()  # stays on device
        self.correct = self.correct + correct
        self.count += output.size(0)

    def update_counts(self, correct, count):
        self.correct = self.correct + correct
        self.count += count

    @property
    def accuracy(self):
        return _to_float(self.correct) / max(self.count, 1)

    def __str__(self):
        return '{:.2f}%'.format(self.accuracy * 100)
