"""BASELINE.json config 1: ResNet-18 / CIFAR-10-shape, world_size = 1, on the CPU (plumbing run).

Drives the eager ``Trainer`` (the reference's train-loop API, `pytorch_collab.py:36-249`) through
its own step function on synthetic CIFAR-10-shaped data (no dataset download offline) and
prints one JSON line: trained images/s, ms/step, and the share of the step spent scoring the
presample pool.  ``--uniform`` is the config as written (uniform-sample training, no scoring
pass); the default is the reference's importance-sampled step, whose CPU rate BASELINE.md
measured at 39-43 trained img/s on this container.

    python examples/cpu_reference_step.py [--uniform] [--optimizer sgd] [--steps 10]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--uniform', action='store_true', help='uniform sampling (no scoring pass)')
    ap.add_argument('--optimizer', default='sgd', choices=('sgd', 'adam'))
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--threads', type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    import torch
    from mercury_amd.collab import make_optimizer
    from mercury_amd.config import Config
    from mercury_amd.data import load_cifar10_noniid
    from mercury_amd.models import ResNet18
    from mercury_amd.trainer import Trainer
    from mercury_amd.utils.meters import Accuracy, Average, EMAverage
    if args.threads:
        torch.set_num_threads(args.threads)
    cfg = Config(importance=not args.uniform, optimizer=args.optimizer, print_every=0,
                 eval_every=0, engine='eager')
    np.random.seed(cfg.seed)
    pres, train, test = load_cifar10_noniid(1, cfg.dirichlet_alpha, cfg.batch_size,
                                            data_dir='/nonexistent')   # synthetic fallback
    torch.manual_seed(0)
    net = ResNet18(10)
    t = Trainer(net, make_optimizer(cfg, net.parameters(), 1), train, pres[0], test, 'cpu', cfg)
    loss, acc, ema = Average(), Accuracy(), EMAverage(cfg.ema_alpha)
    batch = t.update_samples(ema)
    for i in range(args.warmup + args.steps):
        if i == args.warmup:
            t.timer.collect()                  # drop warmup phase times
            t0 = time.perf_counter()
        # Trainer.train_step = IS-weighted fwd/bwd + next update_samples (the scoring pass) +
        # average_gradients + optimizer step; the PhaseTimer splits the phases
        batch, _ = t.train_step(*batch[:3], ema, loss, acc)
    dt = time.perf_counter() - t0
    phases = t.timer.collect()                 # mean ms per step and phase
    t_score = phases.get('score', 0.0) * args.steps / 1e3
    out = {'metric': 'trained images/s (CPU plumbing run, BASELINE config 1)',
           'value': round(cfg.batch_size * args.steps / dt, 2), 'unit': 'trained images/s',
           'ms_per_step': round(dt * 1e3 / args.steps, 2), 'n_gpus': 0, 'steps': args.steps,
           'sampler': 'uniform' if args.uniform else 'importance (loss + 0.5*EMA)',
           'scoring_share_pct': round(100 * t_score / dt, 1) if t_score else None,
           'phases_ms': {k: round(v, 2) for k, v in phases.items()},
           'optimizer': args.optimizer, 'threads': torch.get_num_threads(), 'dtype': 'fp32',
           'data': 'synthetic', 'final_loss': round(float(loss.average), 4)}
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
