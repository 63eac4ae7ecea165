"""Flatten / unflatten of nested tensor lists (`util.py:12-63`).

The reference copies every gradient into a fresh concatenated buffer on every
step (`pytorch_collab.py:240`) and slices it back.  These helpers keep that API
for compatibility, but the DP engine (``mercury_amd.parallel.flat``) never calls
them on the hot path: parameters and gradients live in one persistent flat
buffer and the per-tensor tensors are views into it.
"""
from __future__ import annotations

import numpy as np
import torch


def _flatten(values):
    if isinstance(values, np.ndarray) or torch.is_tensor(values):
        yield values.reshape(-1)
    else:
        for value in values:
            yield from _flatten(value)


def flatten(values):
    """Nested lists of ndarray -> 1-D ndarray."""
    return np.concatenate(list(_flatten(values)))


def flatten_torch_tensor(values):
    """Nested lists of tensors -> 1-D tensor (copy)."""
    return torch.cat(list(_flatten(values)), 0)


def _unflatten(flat_values, prototype, offset):
    if isinstance(prototype, np.ndarray) or torch.is_tensor(prototype):
        shape = prototype.shape
        n = int(np.prod(shape)) if len(shape) else 1
        value = flat_values[offset:offset + n].reshape(shape)
        return value, offset + n
    result = []
    for value in prototype:
        value, offset = _unflatten(flat_values, value, offset)
        result.append(value)
    return result, offset


def unflatten(flat_values, prototype):
    """1-D array -> nested list with the structure of ``prototype`` (views)."""
    result, offset = _unflatten(flat_values, prototype, 0)
    assert offset == len(flat_values)
    return result


def unflatten_torch_tensor(flat_values, prototype):
    """1-D tensor -> nested list with the structure of ``prototype`` (views)."""
    result, offset = _unflatten(flat_values, prototype, 0)
    assert offset == flat_values.numel()
    return result
