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


@dataclass
class EngineOptions:
    """Kernel-path switches of the native engine (``engine/native.py``).

    The defaults are the measured-best paths; every field names the same-box A/B that keeps
    it (``profiles/``).  Set them in code (``NativeEngine(..., opts=EngineOptions(...))``) or,
    for A/B runs of an unmodified tree, with ONE environment variable parsed by ``from_env``:

        MERCURY_ENGINE_OPTS="hconv=score,pgemm=0,hconv_plans=32,16,128,128=64,64,1"

    (items separated by ',' where the next item starts with ``name=``)."""
    # stride-1 3x3 convs on the halo-tile kernel: '1' both batch modes, 'score' / 'train' one,
    # '0' igemm everywhere (profiles/r2/ab_hconv_modes.json, ab_train_persist.json)
    hconv: str = '1'
    # persistent halo-kernel plans ('0' per-tile plans only; profiles/r2/ab_hconv_persistent.json)
    hconv_persist: bool = True
    # persistent halo-kernel grid (0: half the CUs -- the scoring convs run beside the train
    # stream; 256 blocks 1.653, 128 1.525 ms/step, profiles/r2/ab_hconv_persistent.json)
    hconv_persist_grid: int = 0
    # waves per persistent halo block (8: 1.513 vs 1.521 ms/step over 4)
    hconv_persist_waves: int = 8
    # 8-wave layout of the 128 x 64 persistent tile: wave rows (8 = 8 x 1, 16 x 64 per wave,
    # every wave reading the whole weight tile; 4 = 4 x 2, 32 x 32 per wave, 20 % fewer LDS
    # fragment bytes per MFMA: layer3 scoring conv 57.5-58.1 vs 60.2-61.5 us, scoring solo
    # 1.034-1.036 vs 1.041-1.046 ms, step within noise, profiles/r6/ab_r6a/)
    hconv_persist_wm8: int = 4
    # per-tile halo kernel: the row-term halo swizzle (HconvGeom.SWA) where the lane-group model
    # finds it conflict-free (layer4: 2.03 -> 0.08 LDS conflict cycles per LDS instruction)
    hconv_swa: bool = True
    # ResNet-50's stride-1 3x3 convs on the persistent halo kernel with padded row tiles where
    # measured faster (hconv.MEASURED_PAD; 56-/28-wide images have no whole-row 128/256 tile)
    hconv_pad: bool = True
    # forward convs with the BN-apply prologue on their measured split-K plans
    # (ops.conv.MEASURED_PRO; MobileNetV2's train-batch project convs)
    pro_plans: bool = True
    # stride-1 3x3 convs on the row-step persistent kernel (csrc/hconv.hip hrow_kernel) where it
    # measured faster: '1' both batch modes, 'score' / 'train' one, '0' off (hconv.MEASURED_ROW;
    # layer1 scoring conv 51.6 vs 60.4 us, profiles/r5/hrow_bench_v3.jsonl)
    hconv_row: str = 'score'
    # per-shape halo plan overrides for sweeps: "N,H,C,K=bm,bn,splits;..." ('none' = igemm)
    hconv_plans: str = ''
    # 1x1 convs on the persistent LDS-DMA pointwise GEMM (profiles/r3/pgemm_cmp_v2.jsonl)
    pgemm: bool = True
    # narrow-input expansion 1x1 convs on the panel-resident kernel (pwconv_engine_ab.json)
    pwconv: bool = True
    # plain (no prologue) narrow-input expansion 1x1 convs on the panel-resident kernel too
    # (ResNet-50 layer1.0 shortcut; ops.conv.pwconv_plain_wins)
    pwconv_plain: bool = True
    # first conv on the dense-k stem kernel (stem_bench_v2.jsonl)
    stem: bool = True
    # a downsampling block's first conv and its shortcut conv in one launch (profiles/r4/
    # ab_dual_fwd.json)
    dual_fwd: bool = True
    # priority of the scoring / comm streams (ops.role_stream): '0' default, '-1' high, 'auto'
    # = high under DP, default otherwise.  A high-priority scoring queue is dispatched ahead of
    # the critical train chain (MobileNetV2 2.78 vs 2.93 ms, VGG11 3.82 vs 4.10, ResNet-18
    # neutral, profiles/r4/ab_stream_prio.json); but once RCCL has created its streams, only
    # the high-priority pool gives the role streams queues of their own (forced DP 2.79 ms on
    # default-priority role streams, profiles/r4/session_r4s26/)
    role_prio: str = 'auto'
    # the shortcut's backward pair in one launch with the block's last conv's pair (profiles/r4/
    # ab_dual_bwd.json)
    dual_bwd: bool = True
    # intra-block BN + activation folded into the consuming conv's operand load
    fuse_bn_fwd: bool = True
    # block-final BN + identity residual in the next block's pointwise conv load (ab_res_pro.json)
    res_pro: bool = True
    # depthwise convs take their input's BN + activation in their loads (MobileNetV2)
    dw_pro: bool = True
    # depthwise dgrad + wgrad in one launch, wgrad reduces batched (ab_dw_pair.json)
    dw_pair: bool = True
    # the classifier head's backward reduces the final BN's backward sums (ab_head_bw.json)
    head_bw: bool = True
    # stride-2 dgrad as four parity classes (ab_dgrad_s2.json)
    dgrad_s2: bool = True
    # one-launch optimizer that also writes the bf16 weight copies (bench_fused_opt_r2h.json)
    fused_opt: bool = True
    # the DP train phase as ONE executable graph (the segment graphs chained as child nodes) with
    # an event-record node after each bucket's segment; the host issues each bucket's all-reduce
    # on the comm stream behind its node (no graph-internal comm streams;
    # profiles/r4/ab_comm_events.json)
    comm_events: bool = True
    # issue the RCCL all-reduce even on a one-rank communicator (forced buckets at W = 1; it is
    # the identity there -- the tests exercise RCCL with it, the bench measures without)
    rccl_one_rank: bool = False
    # scoring / eval: the last block's BN (+ identity residual) + activation applied by the
    # classifier head's average pool instead of a bn_apply pass over the last activation
    head_bn: bool = True
    # DP bucket plan from a start-up timing of the engine's RCCL all-reduce (parallel/buckets.py
    # calibrate_allreduce): 'auto' when the engine chose the bucket size (W > 1, or W = 1 with
    # rccl_one_rank), 'on' always (an explicit bucket_bytes still wins; the last-bucket size is
    # taken from the calibration), 'off' never (16 MiB buckets, 1 MiB last bucket)
    bucket_calib: str = 'auto'
    # the last DP bucket's budget in MiB when nothing was calibrated (0: no forced last-bucket
    # cut -- the 16 MiB walk decides alone)
    last_bucket_mb: float = 1.0
    # scoring-pass conv tile target in blocks (128 vs 256: 1.656 vs 1.667 ms/step)
    score_min_blocks: int = 128
    # debug mode: print each phase as it completes
    debug_log: bool = False
    # the scoring pass's intra-block BN + activation applied in the halo staging of the
    # persistent convs, no bn_apply pass: '1' every persistent conv, 'row' only the row-step
    # kernel's (hconv_row), '0' none.  On the per-tap kernel the staging transform costs more
    # than the pass it saves (layer3 81.5 vs 57 us): 'row' 1.307 vs '1' 1.333 ms/step with the
    # layer1 + layer2 convs on the row-step kernel (profiles/r5/ab_persist_bn_scope.json)
    # ('stat': the row-step kernel's weight-stationary layer1 convs only)
    persist_bn: str = 'row'

    @classmethod
    def from_env(cls, base=None):
        import os
        import re
        o = dataclasses.replace(base) if base is not None else cls()
        spec = os.environ.get('MERCURY_ENGINE_OPTS', '').strip()
        if not spec:
            return o
        types = {f.name: f.type for f in dataclasses.fields(cls)}
        for item in re.split(r',(?=[a-z_][a-z0-9_]*=)', spec):
            if '=' not in item:
                raise ValueError('MERCURY_ENGINE_OPTS: %r is not name=value' % item)
            k, v = item.split('=', 1)
            k = k.strip()
            if k not in types:
                raise ValueError('MERCURY_ENGINE_OPTS: unknown option %r (EngineOptions)' % k)
            t = types[k]
            if t in ('bool', bool):
                val = v.strip().lower() in ('1', 'true', 'yes', 'on')
            elif t in ('int', int):
                val = int(v)
            elif t in ('float', float):
                val = float(v)
            else:
                val = v.strip()
            setattr(o, k, val)
        return o

