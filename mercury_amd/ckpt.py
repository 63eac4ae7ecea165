"""Checkpoint / resume with a reference-compatible layout.

The reference never saves anything; compatibility is therefore defined as:

(a) ``model`` is a plain ``state_dict`` whose keys and shapes equal the
    reference ``nn.Module``'s (ResNet-18: 122 keys), in PyTorch's NCHW/KCRS
    fp32 layout -- the native engine converts its flat NHWC/bf16 state back on
    save, so the file loads into ``pytorch_model.ResNet18(10)`` directly;
(b) ``optimizer`` / ``scheduler`` are torch ``state_dict``s;
(c) sampler state uses the reference field names: ``step``, ``epoch``, EMA
    ``{first_update, value, alpha}`` (`util.py:202-205`) and, if present, the
    ``Groupwise_Sampler`` fields (`util.py:106-112`);
(d) ``net_dataidx_map`` -- this rank's partition (`data_loader.py:126-173`).

Everything is saved with tensors / numbers / lists only, and loaded with
``torch.load(weights_only=True)``.
"""
from __future__ import annotations

import os

import numpy as np
import torch


def _plain(x):
    if isinstance(x, np.ndarray):
        return torch.from_numpy(np.ascontiguousarray(x))
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    if isinstance(x, np.generic):
        return x.item()
    return x


def checkpoint_dict(trainer, ema=None, sampler=None, net_dataidx_map=None):
    sd = trainer.state_dict()
    out = {'format': 'mercury_amd/1', 'model': sd['model'], 'optimizer': sd['optimizer'],
           'scheduler': sd.get('scheduler'), 'step': int(sd['step']), 'epoch': int(sd['epoch']),
           'epoch_step': int(sd.get('epoch_step', 0))}
    if ema is not None:
        out['ema'] = ema.state_dict()
    if sampler is not None:
        out['sampler'] = _plain(sampler.state_dict())
    if net_dataidx_map is not None:
        out['net_dataidx_map'] = {int(k): torch.as_tensor(np.asarray(v, dtype=np.int64))
                                  for k, v in net_dataidx_map.items()}
    if 'engine' in sd:
        out['engine'] = sd['engine']
    return out


def save_checkpoint(trainer, path, ema=None, sampler=None, net_dataidx_map=None):
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = path + '.tmp'
    torch.save(checkpoint_dict(trainer, ema, sampler, net_dataidx_map), tmp)
    os.replace(tmp, path)  # atomic: a crash never leaves a torn checkpoint
    return path


def resume_path(spec, rank):
    """Per-rank checkpoint file for ``Config.resume``: a path containing ``{rank}`` is
    formatted, a directory resolves to its ``ckpt_rank<r>.pt`` (the name ``Trainer`` writes),
    anything else is used as given (every rank loads the same file)."""
    if '{rank}' in spec:
        return spec.format(rank=rank)
    if os.path.isdir(spec):
        return os.path.join(spec, 'ckpt_rank%d.pt' % rank)
    return spec


def load_checkpoint(trainer, path, ema=None, sampler=None):
    ck = torch.load(path, map_location='cpu', weights_only=True)
    trainer.load_state_dict(ck)
    if ema is not None and 'ema' in ck:
        ema.load_state_dict(ck['ema'])
    if sampler is not None and 'sampler' in ck:
        sampler.load_state_dict({k: (v.numpy() if torch.is_tensor(v) else v)
                                 for k, v in ck['sampler'].items()})
    return ck
