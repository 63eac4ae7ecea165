"""Headline benchmark: importance-sampled ResNet-18 / CIFAR-10-shape DP training.

BASELINE.json metric: "images/sec (whole node) + sampler overhead %, ResNet-18
CIFAR-10 DP 1/2/4/8 GPU".  Each rank runs the reference's default step
(`pytorch_collab.py:127-164`): score a 10x32 = 320-sample presample pool
(forward, ghost-BN per 32), draw 32 samples with replacement proportional to
loss + 0.5*EMA, IS-weighted fwd+bwd on them, gradient all-reduce (RCCL),
Adam.  Per-GPU batch is fixed (weak scaling); ``value`` counts TRAINED images
per second over the whole job (N x 32 x steps / time).  The sampler overhead
is measured in a second timed loop with importance scoring switched off
(uniform 32-sample batches, no pool forward): overhead % = 1 - t_uniform/t_IS.

Data: synthetic CIFAR-10-shaped uint8 images (class-conditional templates +
noise), Dirichlet(0.5) non-IID shards (seed 102) -- no network access for the
real dataset.  Weights are random-init ResNet-18 (11,173,962 params).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
from __future__ import annotations
import os
if int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:   # before torch loads HIP: see
    os.environ['GPU_MAX_HW_QUEUES'] = '16'                # mercury_amd/__init__.py

import argparse
import json
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

REF_CPU_IMG_S = 41.0   # reference step, W=1, 39-43 trained img/s (CPU, only measured number)

HEADLINE = 'images/sec (whole node) + sampler overhead %, ResNet-18 CIFAR-10 DP 1/2/4/8 GPU'
# BASELINE.json configs 2-5 (config 1 is the CPU plumbing run: examples/cpu_reference_step.py)
PRESETS = {
    'resnet18-cifar10': dict(model='resnet18', classes=10, hw=32, n=50000, batch=32,
                             metric=HEADLINE, dataset='cifar10-shape (32x32x3, 10 classes)'),
    'mobilenetv2-cifar100': dict(model='mobilenetv2', classes=100, hw=32, n=50000, batch=32,
                                 metric='images/sec (whole node) + sampler overhead %, '
                                        'MobileNetV2 CIFAR-100 DP',
                                 dataset='cifar100-shape (32x32x3, 100 classes)'),
    'resnet50-imagenet': dict(model='resnet50_imagenet', classes=1000, hw=224, n=12800, batch=128,
                              metric='images/sec (whole node) + sampler overhead %, '
                                     'ResNet-50 ImageNet-shape 224 DP',
                              dataset='imagenet-shape (224x224x3, 1000 classes; 12800 '
                                      'synthetic images resident in HBM)'),
    'vgg11-speech': dict(model='vgg11', classes=30, hw=(101, 161), n=20000, batch=32, chans=1,
                         metric='images/sec (whole node) + sampler overhead %, VGG11 '
                                'speech-commands-shape DP',
                         dataset='GSC-shape spectrograms (1x101x161 float, 30 classes)'),
}


SAMPLER_DESC = {
    'alias': 'importance (loss + 0.5*EMA), with replacement',
    'cdf': 'importance (loss + 0.5*EMA), with replacement (inverse-CDF draws)',
    'groupwise': 'global HBM importance table, current contiguous-slice group, p ~ loss + mean',
}


def preset_data(pre):
    """(image hw, x, y) of a preset: synthetic uint8 images, or float 'spectrograms' (a
    class-dependent low-frequency pattern + noise) for the speech preset."""
    import numpy as np
    from mercury_amd.data.datasets import synthetic_arrays
    ncls, hw, n = pre['classes'], pre['hw'], pre['n']
    hw = hw if isinstance(hw, tuple) else (hw, hw)
    if pre.get('chans', 3) == 3:
        x_all, y_all = synthetic_arrays(n, ncls, shape=(hw[0], hw[1], 3), seed=8)
    else:
        rng = np.random.RandomState(8)
        y_all = rng.randint(0, ncls, n).astype(np.int64)
        proto = rng.randn(ncls, pre['chans'], hw[0], hw[1]).astype(np.float32)
        x_all = (proto[y_all] + rng.randn(n, pre['chans'], hw[0], hw[1]).astype(np.float32) * 2)
    return hw, x_all, y_all


def diagnostics(eng, steps, ws):
    """Untimed steps AFTER the timed loop: device-phase times (HIP events on each stream),
    the DP communicator's view (ranks, bucket bytes, all-reduce device time, the part of it
    not hidden under backward / scoring) and a final replica check across ranks."""
    import torch
    import torch.distributed as dist
    acc = {}
    for _ in range(steps):
        eng.timer.on = True
        eng.step()
        eng.timer.on = False
        ph = eng.timer.collect()
        for k, v in ph.items():
            if not isinstance(v, list):
                acc.setdefault(k, []).append(v)
    med = {k: round(sorted(v)[len(v) // 2], 4) for k, v in acc.items()}
    plan = eng.bucket_plan()
    out = {'device_phase_ms': {k: med[k] for k in ('step', 'critical', 'score', 'train', 'wait',
                                                   'tail') if k in med}}
    dp = {'backend': dist.get_backend() if dist.is_initialized() else None,
          'comm': eng.comm_kind,
          'comm_ranks': eng.comm.size if eng.comm is not None else
          (dist.get_world_size() if dist.is_initialized() else 1),
          'buckets_bytes': [4 * (e - s) for s, e in sorted(plan.values(), reverse=True)],
          'wire': 'ternary' if eng.grad_compress else ('bf16' if eng.wire_bf16 else 'fp32'),
          # one chained train executable with an event node per bucket (timed diag steps:
          # segmented replays)
          'comm_events': bool(eng._train_exec),
          'allreduce_ms_per_step': med.get('comm'), 'comm_exposed_ms': med.get('comm_exposed'),
          'overlap_frac': med.get('overlap'),
          # start-up timing of the engine's RCCL all-reduce and the bucket plan chosen from it
          'calibration': eng.comm_calib,
          # the cross-worker score all-gather on the score stream, device ms
          'score_exchange': eng.score_exchange is not None,
          'global_ema': bool(eng.global_ema and eng.score_exchange is not None),
          'score_allgather_ms_per_step': med.get('score_xchg')}
    if eng.dp and eng.comm is not None and eng.comm.size == 1 and \
            not eng.opts.rccl_one_rank and eng.comm_kind == 'rccl':
        # forced buckets on one GPU: the bucket plan, graph segments, event nodes and comm
        # stream run as at W > 1, but RCCL's one-rank AVG (the identity) is skipped
        dp['collective'] = 'none issued (one-rank AVG skipped; plumbing only)'
    torch.cuda.synchronize()
    if ws > 1:
        # every rank's communicator must span the whole job (one rank per GPU)
        if dp['comm_ranks'] != ws:
            raise RuntimeError('DP communicator spans %s ranks, job has %d'
                               % (dp['comm_ranks'], ws))
        from mercury_amd.parallel.health import check_replicas
        ok, spread = check_replicas(eng.opt.p)
        dp['replicas_identical'] = bool(ok)
        dp['replica_spread'] = float(spread)
    if eng.check_order:
        dp['order_violations'] = eng.order_violations()[0]
    out['dp'] = dp
    if ws == 1 and not eng.dp and eng.graphs:
        out['solo_ms'] = solo_graph_ms(eng)
    return out


def solo_graph_ms(eng, reps=5):
    """Each step graph replayed ALONE (no concurrent stream): how much of the step is
    contention between the scoring and the training stream.  Untimed diagnostic, after the
    timed loop."""
    import torch
    g = eng.graphs

    def t(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return round(e0.elapsed_time(e1) / reps, 4)

    def score():
        g['score'].replay()
        if 'score_sample' in g:
            g['score_sample'].replay()
    return {'score': t(score), 'train': t(lambda: [x.replay() for x, _ in g['train']]),
            'tail': t(lambda: g['tail'].replay())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', default='resnet18-cifar10', choices=sorted(PRESETS))
    ap.add_argument('--batch', type=int, default=0, help='per-GPU batch (0: preset)')
    ap.add_argument('--pool-batches', type=int, default=10)
    ap.add_argument('--no-overhead', action='store_true')
    ap.add_argument('--no-graphs', action='store_true')
    ap.add_argument('--force-buckets', action='store_true',
                    help='issue the RCCL bucket all-reduces even at one GPU (path check)')
    ap.add_argument('--comm', default='auto', choices=('auto', 'rccl', 'xgmi', 'pg'),
                    help='DP all-reduce: own RCCL communicator on a comm stream, the direct-xGMI '
                         'two-shot over IPC-mapped peer buffers, or the torch ProcessGroup')
    ap.add_argument('--wire-bf16', action='store_true', help='bf16 gradients on the wire')
    ap.add_argument('--bucket-mb', type=float, default=0,
                    help='gradient bucket size in MiB (0: the engine default for the world size)')
    ap.add_argument('--compress', default='none', choices=('none', 'ternary'),
                    help='ternary-compressed gradient all-reduce (parallel/compress.py)')
    ap.add_argument('--sampler', default='alias', choices=('alias', 'cdf', 'groupwise'),
                    help="pool draw kernel, or 'groupwise': draws from the HBM importance table "
                         'over the current contiguous-slice group (Groupwise_Sampler)')
    ap.add_argument('--replay-only', choices=('train', 'score'), default=None,
                    help='profiling aid: after warm-up, replay only this step graph --steps '
                         'times (no concurrent stream) and print its time per replay')
    ap.add_argument('--diag-steps', type=int, default=5,
                    help='untimed steps after the timed loop with device-phase events')
    args = ap.parse_args()
    # stdout carries exactly ONE line, the result JSON: everything else written to fd 1 while the
    # job runs (RCCL's version banner at communicator init, library warnings) goes to stderr
    out_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    pre = PRESETS[args.config]
    args.batch = args.batch or pre['batch']

    import numpy as np
    import torch
    import torch.distributed as dist
    from mercury_amd.parallel import dist as pdist
    rank, ws, device = pdist.init_from_env(force=args.force_buckets)
    if ws != args.gpus and rank == 0:
        print('[bench] warning: WORLD_SIZE=%d but --gpus=%d' % (ws, args.gpus), file=sys.stderr)

    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.data.partition import dirichlet_partition
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model

    ncls, n = pre['classes'], pre['n']
    hw, x_all, y_all = preset_data(pre)
    np.random.seed(102)
    shards = dirichlet_partition(y_all, ws, 0.5, ncls) if ws > 1 else {0: np.arange(n)}
    idx = np.asarray(shards[rank])
    torch.manual_seed(1234)
    net = build_model(pre['model'], ncls).to(device)

    def make(importance):
        eng = NativeEngine(net, device, args.batch, args.pool_batches, optimizer='adam',
                           lr=0.001 * ws, seed=7 + rank, importance=importance, world_size=ws,
                           use_graphs=not args.no_graphs, image_hw=hw,
                           force_buckets=args.force_buckets, comm=args.comm,
                           wire_bf16=args.wire_bf16, sampler=args.sampler,
                           bucket_bytes=int(args.bucket_mb * (1 << 20)) or None,
                           grad_compress=args.compress,
                           # under DP the north-star collective runs every step: the pool scores
                           # all-gathered across ranks and one shared EMA normaliser
                           exchange_scores=ws > 1 and args.sampler != 'groupwise',
                           global_ema=ws > 1 and args.sampler != 'groupwise')
        eng.set_shard(x_all[idx], y_all[idx])
        if ws > 1:
            eng.broadcast_from(0)
        return eng

    def run(eng, steps, warmup, scoring=True):
        eng.scoring = scoring
        eng.prime()
        eng.step()
        if eng.use_graphs:
            eng.build_graphs()
        for _ in range(warmup):
            eng.step()
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            eng.step()
        torch.cuda.synchronize()
        if ws > 1:
            dist.barrier()
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
        if ws > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        return float(dt.item())

    eng = make(True)
    if args.replay_only:
        run(eng, 0, args.warmup)
        g = eng.graphs
        rep = (lambda: [x.replay() for x, _ in g['train']]) if args.replay_only == 'train' \
            else (lambda: g['score'].replay())
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rep()
        torch.cuda.synchronize()
        os.write(out_fd, (json.dumps({'replay_only': args.replay_only, 'config': args.config,
                                      'ms_per_replay': round((time.perf_counter() - t0) * 1e3 /
                                                             args.steps, 4)}) + '\n').encode())
        return
    t_is = run(eng, args.steps, args.warmup)
    m = eng.read_meters()
    diag = diagnostics(eng, args.diag_steps, ws)
    ms = t_is * 1e3 / args.steps
    value = ws * args.batch * args.steps / t_is
    overhead = None
    eng_u = None
    if not args.no_overhead:
        eng.close()                      # deterministic teardown before the next engine
        eng_u = make(False)
        t_u = run(eng_u, args.steps, args.warmup, scoring=False)
        overhead = 100.0 * max(0.0, 1.0 - t_u / t_is)
    if rank == 0:
        out = {
            'metric': pre['metric'],
            'value': round(value, 2), 'unit': 'trained images/s', 'n_gpus': ws,
            'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': round(ms, 4),
            'higher_is_better': True, 'scaling': 'weak',
            'vs_baseline': round(value / REF_CPU_IMG_S, 2),
            'baseline_note': 'reference publishes no numbers; BASELINE.md measured its step at '
                             '39-43 trained img/s (W=1, CPU); vs_baseline uses 41',
            'sampler_overhead_pct': None if overhead is None else round(overhead, 2),
            'scored_images_per_sec': round(ws * args.batch * args.pool_batches * args.steps / t_is, 1),
            'dtype': 'bf16', 'data': 'synthetic',
            'config': {'model': pre['model'], 'dataset': pre['dataset'],
                       'global_batch': ws * args.batch, 'per_gpu_batch': args.batch,
                       'presample_pool': args.batch * args.pool_batches, 'seq_len': None,
                       'optimizer': 'adam', 'parallelism': 'dp%d' % ws,
                       'sampler': SAMPLER_DESC[args.sampler]},
            'final_train_loss': round(m['loss_sum'] / max(m['count'], 1), 4),
        }
        out.update(diag)
        sys.stdout.flush()
        os.write(out_fd, (json.dumps(out) + '\n').encode())
    for e in (eng, eng_u):
        if e is not None:
            e.close()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
