"""mercury_amd -- importance-sampled data-parallel training, MI355X-native.

A from-scratch rebuild of the capabilities of AIoT-MLSys-Lab/Mercury
(SenSys'21) for AMD Instinct MI355X (gfx950): hand-written CDNA4 HIP kernels
(``csrc/``) for importance scoring, alias sampling, augmentation and the
ResNet/MobileNet conv/BN stack (MFMA implicit GEMM), RCCL over xGMI for data
parallelism, HIP graphs for the step.  The public train-loop API mirrors the
reference ``pytorch_collab.py`` (see ``mercury_amd.trainer.Trainer``).
"""
import torch  # noqa: F401  (load torch's HIP runtime before our extension)

from .config import Config
from .trainer import Trainer
from . import models, data, importance, parallel, utils

__version__ = '0.1.0'

__all__ = ['Config', 'Trainer', 'models', 'data', 'importance', 'parallel', 'utils']
