"""Launcher: the ``python pytorch_collab.py`` entry point (`pytorch_collab.py:252-292`).

Usage::

    # one process per GPU (preferred; RCCL over xGMI)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m mercury_amd.collab --num-epochs 100
    # reference-style fork launcher (gloo on CPU, or RCCL if there are >= W GPUs)
    python -m mercury_amd.collab --world-size 4

Every rank builds the same Dirichlet partition from ``np.random.seed(seed)``
and keeps its own shard (the reference builds all loaders in the parent and
forks them).  ``my_run`` keeps the reference signature.
"""
from __future__ import annotations
import os
if int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:   # before torch loads HIP: see
    os.environ['GPU_MAX_HW_QUEUES'] = '16'                # mercury_amd/__init__.py

import argparse

import numpy as np
import torch

from .config import Config
from .data.partition import load_cifar10_noniid, load_partition_data_cifar10
from .models import build_model
from .parallel import dist as pdist


def make_optimizer(cfg, params, world_size):
    lr = cfg.lr(world_size)
    if cfg.optimizer == 'sgd':
        return torch.optim.SGD(params, lr=lr, momentum=cfg.momentum,
                               weight_decay=cfg.weight_decay)
    if cfg.optimizer == 'adamw':
        return torch.optim.AdamW(params, lr=lr, weight_decay=cfg.weight_decay)
    return torch.optim.Adam(params, lr=lr, weight_decay=cfg.weight_decay)


def build_loaders(cfg, world_size, rank):
    np.random.seed(cfg.seed)
    if cfg.noniid:
        presam_loaders, train_loader, test_loader = load_cifar10_noniid(
            world_size, cfg.dirichlet_alpha, cfg.batch_size, cfg.data_dir, cfg.dataset)
        return presam_loaders[rank], train_loader, test_loader
    out = load_partition_data_cifar10(cfg.dataset, cfg.data_dir, 'homo', cfg.dirichlet_alpha,
                                      world_size, cfg.batch_size)
    return out[5][rank], out[2], out[3]


def make_trainer(cfg, net, optimizer, train_loader, presam_loader, test_loader, device):
    from .trainer import Trainer
    if cfg.engine in ('native', 'auto') and torch.device(device).type == 'cuda':
        from .engine import native_supported, NativeTrainer
        from .ops.optim import optimizer_spec
        try:
            optimizer_spec(optimizer)
            why = None if native_supported(net) else 'model not supported by the native engine'
        except ValueError as e:
            why = str(e)
        if why is None:
            return NativeTrainer(net, optimizer, train_loader, presam_loader, test_loader,
                                 device, cfg)
        if cfg.engine == 'native':
            raise RuntimeError(why)
        print('[mercury_amd] eager engine: %s' % why, flush=True)
    return Trainer(net, optimizer, train_loader, presam_loader, test_loader, device, cfg)


def my_run(presam_loader, train_loader, test_loader, cfg=None):
    """Build model + optimizer + Trainer and fit (`pytorch_collab.py:252-266`)."""
    cfg = cfg or Config()
    rank, ws = pdist.rank(), pdist.world_size()
    device = torch.device('cuda', torch.cuda.current_device()) if torch.cuda.is_available() \
        else torch.device('cpu')
    torch.manual_seed(cfg.seed + rank)
    net = build_model(cfg.model, cfg.num_classes).to(device)
    if rank == 0:
        print('total parameters', sum(p.numel() for p in net.parameters() if p.requires_grad))
    optimizer = make_optimizer(cfg, net.parameters(), ws)
    trainer = make_trainer(cfg, net, optimizer, train_loader, presam_loader, test_loader, device)
    trainer.fit(cfg.num_epochs)
    return trainer


def _rank_main(rank, world_size, cfg):
    presam, train, test = build_loaders(cfg, world_size, rank)
    my_run(presam, train, test, cfg)


def main(argv=None):
    ap = Config.add_args(argparse.ArgumentParser('mercury_amd.collab'))
    ap.add_argument('--world-size', type=int, default=0)
    ns = ap.parse_args(argv)
    cfg = Config(**{k: v for k, v in vars(ns).items() if k in Config.__dataclass_fields__})
    if 'WORLD_SIZE' in os.environ:  # torchrun: one process per GPU
        rank, ws, device = pdist.init_from_env()
        _rank_main(rank, ws, cfg)
        if pdist.is_initialized():
            torch.distributed.destroy_process_group()
        return
    ws = ns.world_size or 1
    if ws == 1:
        _rank_main(0, 1, cfg)
        return
    backend = 'nccl' if torch.cuda.is_available() and torch.cuda.device_count() >= ws else 'gloo'
    pdist.spawn(_rank_main, ws, args=(cfg,), backend=backend)


if __name__ == '__main__':
    main()
