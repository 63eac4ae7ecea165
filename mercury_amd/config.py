"""Run configuration: one dataclass whose defaults are the reference literals.

Reference constants are scattered over `pytorch_collab.py:21-33` (alpha, seed,
world size, epochs, lr = 0.001*W, log dir), `exp_dataset.py:11-16` (batch 32,
'hetero', ./data/cifar10), `pytorch_collab.py:95` (10 presample batches),
`pytorch_collab.py:170,181` (print/eval cadence 100/200) and `util.py:202`
(EMA 0.9).  ``Config.from_args`` builds a CLI with one flag per field.
"""
from __future__ import annotations

import argparse
import dataclasses
import time
from dataclasses import dataclass


@dataclass
class Config:
    # importance sampling
    alpha: float = 0.5              # IS smoothing: p ~ loss + alpha*EMA
    ema_alpha: float = 0.9          # EMAverage decay
    presample_batches: int = 10     # pool = presample_batches * batch_size
    importance: bool = True         # False -> uniform sampling baseline
    global_ema: bool = False        # share the EMA normaliser across ranks (score all-gather)
    exchange_scores: bool = False   # all-gather pool scores every step (global importance view)
    score: str = 'loss'             # importance score: 'loss' (reference) | 'gradnorm' (per-sample
                                    # classifier-layer gradient norm)
    sampler: str = 'alias'          # 'alias' (Walker table) | 'cdf' (inverse CDF) | 'groupwise'
    #                                 (draws from the HBM importance table, Groupwise_Sampler)
    # data
    dataset: str = 'cifar10'
    data_dir: str = './data/cifar10'
    num_classes: int = 10
    noniid: bool = True
    partition: str = 'hetero'
    dirichlet_alpha: float = 0.5
    batch_size: int = 32
    image_size: int = 32
    # model / optimisation
    model: str = 'resnet18'
    optimizer: str = 'adam'
    base_lr: float = 0.001          # lr = base_lr * world_size (linear scaling)
    momentum: float = 0.9
    weight_decay: float = 0.0
    num_epochs: int = 100
    max_samples: int = 10_000_000   # `fit` stops once step*W exceeds this
    seed: int = 102
    # engine
    engine: str = 'auto'            # 'native' (MI355X kernels + HIP graphs) | 'eager' | 'auto'
    parity: bool = False            # reference quirks: per-param init all-reduce, 10 separate scoring forwards
    bucket_mb: float = 0.0          # 0 -> default_bucket_bytes(W)
    wire_bf16: bool = False         # bf16 gradient all-reduce
    grad_compress: str = 'none'     # 'ternary': stochastic 2-bit gradient wire (quantize_tensor,
                                    # util.py:65-70; parallel/compress.py), native DP path
    overlap: bool = True            # scoring of step t+1 overlaps backward/all-reduce of step t
    use_graphs: bool = True
    comm: str = 'auto'              # native DP all-reduce: 'rccl' (own communicator + comm stream),
                                    # 'xgmi' (direct two-shot over IPC-mapped peer buffers),
                                    # 'pg' (torch ProcessGroup), 'auto' (rccl on nccl backends)
    force_buckets: bool = False     # issue the bucket all-reduces even at world size 1
    # debug / race detection
    debug: bool = False             # serialise streams, no graphs, sync + check after every phase
    check_order: bool = False       # device-side stream-order assertions every step
    # logging
    print_every: int = 100
    eval_every: int = 200           # 0 disables evaluation inside train()
    eval_all_ranks: bool = False
    log_dir: str = ''
    log_str: str = 'ow_ub'
    checkpoint_dir: str = ''
    checkpoint_every: int = 0
    resume: str = ''
    # observability / health
    check_replicas_every: int = 0   # DP replica fingerprint compare cadence (0 = off)
    replica_rtol: float = 0.0       # allowed relative spread (0: bit-identical)
    on_divergence: str = 'raise'    # 'raise' | 'warn'
    roctx: bool = False             # per-phase roctx ranges (rocprofv3 --marker-trace)
    profile_start: int = 0          # step at which the 'mercury_profile' roctx window opens
    profile_steps: int = 0          # window length (0 = off)

    def lr(self, world_size):
        return self.base_lr * world_size

    def pool_size(self):
        return self.presample_batches * self.batch_size

    def default_log_dir(self, world_size):
        return 'trial/cifar10collab_sgd/{}_alpha{}_s{}_{}_lr{}_seed{}{}'.format(
            self.log_str, self.alpha, world_size, self.model, self.lr(world_size), self.seed,
            time.strftime('%m-%d-%H_%M'))

    @classmethod
    def add_args(cls, parser):
        for f in dataclasses.fields(cls):
            name = '--' + f.name.replace('_', '-')
            if f.type in ('bool', bool):
                parser.add_argument(name, type=lambda s: s.lower() in ('1', 'true', 'yes', 'y'),
                                    default=f.default)
            else:
                typ = {'int': int, 'float': float, 'str': str}.get(f.type, type(f.default))
                parser.add_argument(name, type=typ, default=f.default)
        return parser

    @classmethod
    def from_args(cls, argv=None):
        p = cls.add_args(argparse.ArgumentParser('mercury_amd'))
        ns, _ = p.parse_known_args(argv)
        return cls(**{f.name: getattr(ns, f.name) for f in dataclasses.fields(cls)})

    def to_dict(self):
        return dataclasses.asdict(self)

