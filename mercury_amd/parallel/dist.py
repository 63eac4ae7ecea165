"""Process-group setup: one process per GPU, RCCL over xGMI (`pytorch_collab.py:269-292`).

The reference forks W processes that all share GPU 0 and talk gloo over TCP
with an invalid port.  Here:

* ``init_from_env`` reads torchrun's ``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*``,
  pins ``LOCAL_RANK`` to its own GPU and initialises ``backend='nccl'`` (RCCL
  on ROCm) -- or gloo on CPU;
* ``init_processes`` keeps the reference signature for the fork-style launcher;
* ``spawn`` is the reference launcher (W local processes) with exit-code
  propagation: if any rank fails the others are terminated and the error is
  raised (the reference ``join``s without checking);
* every process group gets a timeout so a dead peer cannot hang the job.
"""
from __future__ import annotations

import datetime
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

DEFAULT_TIMEOUT_S = int(os.environ.get('MERCURY_PG_TIMEOUT', '600'))


def free_port():
    """A free TCP port for a local rendezvous, drawn BELOW the kernel's ephemeral range
    (32768-60999): a port the OS hands out for binding 0 is one any other socket (an RCCL / gloo
    connection of a neighbouring test, the TCPStore clients) may be given before rank 0 listens on
    it -- a 2-rank GPU test once failed with EADDRINUSE that way."""
    import random
    rng = random.Random()
    for _ in range(64):
        p = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(('127.0.0.1', p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def is_initialized():
    return dist.is_available() and dist.is_initialized()


def rank():
    return dist.get_rank() if is_initialized() else 0


def world_size():
    return dist.get_world_size() if is_initialized() else 1


def default_backend(device):
    return 'nccl' if torch.device(device).type == 'cuda' else 'gloo'


def init_from_env(device=None, backend=None, timeout_s=DEFAULT_TIMEOUT_S, force=False):
    """Initialise from torchrun env vars; returns ``(rank, world_size, device)``.

    Works without any env (single process) -- then no process group is made unless ``force``
    (a one-rank group, so the collective code paths run on one GPU)."""
    ws = int(os.environ.get('WORLD_SIZE', '1'))
    rk = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', str(rk)))
    if device is None:
        device = 'cuda' if torch.cuda.is_available() else 'cpu'
    device = torch.device(device)
    if device.type == 'cuda':
        torch.cuda.set_device(local)
        device = torch.device('cuda', local)
    if (ws > 1 or force) and not is_initialized():
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29500')
        kw = {}
        if device.type == 'cuda':
            kw['device_id'] = device
        dist.init_process_group(backend or default_backend(device), rank=rk, world_size=ws,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return rk, ws, device


def init_processes(rank, size, presam_loader, train_loader, test_loader, fn, backend='gloo',
                   master_port=None):
    """Reference-signature initialiser (`pytorch_collab.py:269-276`)."""
    os.environ['MASTER_ADDR'] = os.environ.get('MASTER_ADDR', '127.0.0.1')
    os.environ['MASTER_PORT'] = str(master_port or os.environ.get('MASTER_PORT', '29500'))
    os.environ['RANK'] = str(rank)
    os.environ['WORLD_SIZE'] = str(size)
    os.environ.setdefault('LOCAL_RANK', str(rank))
    if backend == 'nccl' and torch.cuda.is_available():
        torch.cuda.set_device(rank % torch.cuda.device_count())
    dist.init_process_group(backend, rank=rank, world_size=size,
                            timeout=datetime.timedelta(seconds=DEFAULT_TIMEOUT_S))
    try:
        return fn(presam_loader, train_loader, test_loader)
    finally:
        dist.destroy_process_group()


def _entry(rank, size, port, backend, fn, args):
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['RANK'] = str(rank)
    os.environ['WORLD_SIZE'] = str(size)
    os.environ['LOCAL_RANK'] = str(rank)
    if backend == 'nccl':
        torch.cuda.set_device(rank)
    dist.init_process_group(backend, rank=rank, world_size=size,
                            timeout=datetime.timedelta(seconds=DEFAULT_TIMEOUT_S))
    try:
        fn(rank, size, *args)
    finally:
        dist.destroy_process_group()


def spawn(fn, world_size, args=(), backend='gloo'):
    """Run ``fn(rank, world_size, *args)`` in W processes; raises if any rank fails.

    ``torch.multiprocessing.spawn`` already terminates the survivors when one
    rank exits non-zero, which is the watchdog behaviour we want."""
    port = free_port()
    mp.spawn(_entry, args=(world_size, port, backend, fn, args), nprocs=world_size, join=True)
