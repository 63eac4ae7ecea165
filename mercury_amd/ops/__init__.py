"""Python front-end for the CDNA4 HIP kernels in ``csrc/``.

Each wrapper validates shapes / dtypes / devices / contiguity and then calls the
raw launcher in ``mercury_amd._C`` on the *current* HIP stream (so every call
is capturable into a HIP graph).  There is no silent fallback: on a machine
with a GPU, a missing or stale extension raises.  The plain-PyTorch fp32
oracles the kernels are tested against live in ``tests/refutil.py`` and in each
GPU test; the CPU path is the eager ``mercury_amd.trainer.Trainer``.

Layout conventions: activations NHWC bf16 with channels padded to a multiple
of 8; conv weights bf16 [K][R][S][Cpad] (forward) and [C][R][S][K] (dgrad);
gradients and optimizer state fp32.
"""
from __future__ import annotations

import importlib
import importlib.util
import os

import torch

_lib = None
_err = None


def lib():
    """The loaded extension; builds it in-tree on first use if absent."""
    global _lib, _err
    if _lib is not None:
        return _lib
    alt = os.environ.get('MERCURY_EXT_PATH')
    if alt:   # A/B builds: another build of the same extension (bench/build_variant.py)
        spec = importlib.util.spec_from_file_location('mercury_amd._C', alt)
        _lib = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(_lib)
        return _lib
    try:
        _lib = importlib.import_module('mercury_amd._C')
    except ImportError as e:  # try an in-tree build (hipcc is in the image)
        _err = e
        if os.environ.get('MERCURY_NO_AUTOBUILD'):
            raise
        from .. import _build
        _build.build(verbose=True)
        _lib = importlib.import_module('mercury_amd._C')
    return _lib


def available():
    try:
        lib()
        return torch.cuda.is_available()
    except Exception:
        return False


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream


_ROLE_STREAMS = {}


def role_stream(device, role, priority=0):
    """The process-wide stream of ``role`` ('score', 'comm') on ``device``, shared by every
    engine of the process.

    HIP runs each stream on one of GPU_MAX_HW_QUEUES hardware queues PER PRIORITY and, past
    that many streams, makes a new stream share the least-used queue of its priority; two
    streams on one queue run back to back.  PyTorch hands out its pooled streams round-robin,
    so with the 4 queues the boxes export an engine's scoring stream could land on the train
    stream's queue and run its step serially (1.37 -> 2.1-2.2 ms, bench/queue_probe.py,
    profiles/r4/queue_probe.json).  The package raises GPU_MAX_HW_QUEUES to 16 before HIP
    starts, and the role streams are taken once, consecutively, and cached per process.
    ``priority`` (EngineOptions.role_prio) 0 takes them from the default-priority pool: a
    HIGH-priority (-1) scoring queue is dispatched ahead of the critical train chain
    (MobileNetV2 2.93 vs 2.78 ms, VGG11 4.10 vs 3.82, profiles/r4/ab_stream_prio.json); but
    once RCCL has created its own streams, default-priority role streams shared queues again
    (forced DP 2.79 vs 1.44 ms), so DP engines take -1 (EngineOptions.role_prio 'auto').  (A
    CU-masked stream gets an unpooled queue but measured serial: 2.26 ms/step.)"""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    key = (idx, int(priority))
    if key not in _ROLE_STREAMS:
        d = torch.device('cuda', idx)
        _ROLE_STREAMS[key] = {r: torch.cuda.Stream(d, priority=int(priority))
                              for r in ('score', 'comm')}
    return _ROLE_STREAMS[key][role]


def ptr(t):
    return 0 if t is None else t.data_ptr()


def _chk(t, dtype, name, numel=None):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError('%s must be a HIP device tensor' % name)
    if t.dtype != dtype:
        raise TypeError('%s: expected %s, got %s' % (name, dtype, t.dtype))
    if not t.is_contiguous():
        raise ValueError('%s must be contiguous' % name)
    if numel is not None and t.numel() < numel:
        raise ValueError('%s too small: %d < %d' % (name, t.numel(), numel))


from .conv import (ConvSpec, conv_fwd, conv_fwd_dual, conv_dgrad, conv_wgrad, conv_bwd, pick_tiles, pack_conv_weight,  # noqa: E402
                   to_nhwc, from_nhwc, pgemm_fwd, pwconv_fwd, stem_fwd)
from .bn import bn_apply, bn_bwd, BnRunTable, sums_numel, sums_total  # noqa: E402
from .head import head_fwd, head_bwd, mlp_head_fwd, mlp_head_bwd  # noqa: E402
from .importance import pool_build, is_sample, gather  # noqa: E402
from .table import ImportanceTable  # noqa: E402
from .optim import FlatOptimizer, optimizer_spec  # noqa: E402
from .misc import (quantize, pool2d_fwd, maxpool2d_bwd, dwconv_fwd, dwconv_dgrad, dwconv_wgrad, dwconv_wgrad_slab_floats,
                   dwconv_bwd, dwconv_wgrad_reduce_batch, dwconv_wgrad_blocks,  # noqa: E402
                   nchw_to_nhwc8, tern_pack, tern_unpack)

__all__ = ['lib', 'available', 'ConvSpec', 'conv_fwd', 'conv_fwd_dual', 'pgemm_fwd', 'pwconv_fwd', 'stem_fwd', 'conv_dgrad', 'conv_wgrad', 'conv_bwd', 'pick_tiles',
           'pack_conv_weight', 'to_nhwc', 'from_nhwc', 'bn_apply', 'bn_bwd', 'BnRunTable', 'sums_numel', 'sums_total',
           'head_fwd', 'head_bwd', 'mlp_head_fwd', 'mlp_head_bwd', 'pool_build', 'is_sample', 'gather', 'ImportanceTable',
           'FlatOptimizer', 'optimizer_spec', 'quantize', 'tern_pack', 'tern_unpack', 'pool2d_fwd', 'maxpool2d_bwd',
           'dwconv_fwd', 'dwconv_dgrad', 'dwconv_wgrad', 'dwconv_wgrad_slab_floats',
           'dwconv_bwd', 'dwconv_wgrad_reduce_batch', 'dwconv_wgrad_blocks',
           'nchw_to_nhwc8']
