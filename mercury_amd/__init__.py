"""mercury_amd -- importance-sampled data-parallel training, MI355X-native.

A from-scratch rebuild of the capabilities of AIoT-MLSys-Lab/Mercury
(SenSys'21) for AMD Instinct MI355X (gfx950): hand-written CDNA4 HIP kernels
(``csrc/``) for importance scoring, alias sampling, augmentation and the
ResNet/MobileNet conv/BN stack (MFMA implicit GEMM), RCCL over xGMI for data
parallelism, HIP graphs for the step.  The public train-loop API mirrors the
reference ``pytorch_collab.py`` (see ``mercury_amd.trainer.Trainer``).
"""
import os

# HIP runs every stream on one of GPU_MAX_HW_QUEUES hardware queues PER PRIORITY (4 by default)
# and makes a stream created past that count SHARE the least-used queue; two streams on one queue
# run back to back.  The engine's step needs its train, scoring and comm streams to overlap, and
# RCCL and PyTorch's stream pools create streams of their own, so with 4 queues the comm stream
# of a DP engine landed on a queue with other work and the step ran serially (ResNet-18 forced
# DP at W=1: 2.25-2.29 ms with 4 or 8 queues, 1.477 with 16, in the process order a DP program
# uses; bench/dist_probe.py, profiles/r4/ab_hw_queues.json).  Set it before the HIP runtime
# starts (before `import torch` to be safe): it takes effect only when mercury_amd is imported first
# (bench.py, collab.py and tests/conftest.py set it first thing; a DP program of your own should
# export GPU_MAX_HW_QUEUES=16).  Raised, not defaulted: the MI355X boxes export the HIP default
# (4) explicitly, which a setdefault would keep (profiles/r4/ab_hw_queues.json).
# MERCURY_KEEP_HW_QUEUES=1 opts out.  ``HW_QUEUES`` records what happened; NativeEngine warns
# once when the raise could not take effect (HIP was already initialised at import).
import sys  # noqa: E402
import warnings  # noqa: E402

HW_QUEUES = {'before': os.environ.get('GPU_MAX_HW_QUEUES'), 'raised': False, 'effective': True}
_hip_up = 'torch' in sys.modules and sys.modules['torch'].cuda.is_initialized()
if os.environ.get('MERCURY_KEEP_HW_QUEUES', '0') != '1' and \
        int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:
    before = HW_QUEUES['before']
    if before not in (None, '', '4'):
        # (4 is HIP's own default, which the MI355X boxes export explicitly)
        warnings.warn('mercury_amd: raising GPU_MAX_HW_QUEUES from %s to 16 (the step overlaps '
                      'three streams; set MERCURY_KEEP_HW_QUEUES=1 to keep yours)' % before,
                      RuntimeWarning, stacklevel=2)
    os.environ['GPU_MAX_HW_QUEUES'] = '16'
    HW_QUEUES['raised'] = True
    HW_QUEUES['effective'] = not _hip_up
elif int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:
    HW_QUEUES['effective'] = False
del _hip_up

import torch  # noqa: F401,E402  (load torch's HIP runtime before our extension)

from .config import Config  # noqa: E402
from .trainer import Trainer  # noqa: E402
from . import models, data, importance, parallel, utils  # noqa: E402

__version__ = '0.1.0'

__all__ = ['Config', 'Trainer', 'models', 'data', 'importance', 'parallel', 'utils']
