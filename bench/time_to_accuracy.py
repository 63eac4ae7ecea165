"""Time-to-accuracy: importance sampling vs uniform sampling (Mercury's actual claim).

Mercury trades per-step throughput (every step also scores a 10x32 pool) for
fewer steps to a target accuracy.  This runs the native engine twice on the
same synthetic CIFAR-10-shaped shard, same init, same Adam -- once with the
reference importance sampler, once uniform -- evaluates held-out accuracy
every ``--eval-every`` steps, and reports steps and wall time (event-timed
train steps only, evaluation excluded) to reach ``--target``.

The synthetic task (low-contrast class templates under pixel noise, plus a fraction of
relabelled "hard" samples) is NOT CIFAR-10, so the numbers measure the
mechanism, not the paper's accuracy curve (no dataset download is possible).

    python bench/time_to_accuracy.py [--steps 3000] [--target 0.8] > tta.json
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def make_data(n, ncls, seed, noise, hard_frac, contrast):
    """Low-contrast class templates under pixel noise: x = 128 + contrast*(t_y - 128) + noise."""
    from mercury_amd.data.datasets import synthetic_arrays
    x, y = synthetic_arrays(n, ncls, seed=seed, noise=0)
    rng = np.random.RandomState(seed + 1)
    xf = 128.0 + contrast * (x.astype(np.float32) - 128.0)
    xf += rng.randint(-noise, noise + 1, size=x.shape).astype(np.float32)
    x, y = np.clip(xf, 0, 255).astype(np.uint8), y.copy()
    hard = rng.rand(n) < hard_frac          # label noise: a minority of confusing samples
    y[hard] = rng.randint(0, ncls, hard.sum())
    return x, y


def run(importance, args, xtr, ytr, xte, yte):
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    torch.manual_seed(args.seed)
    net = build_model(args.model, 10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, lr=args.lr, seed=11, importance=importance,
                       use_graphs=True)
    eng.set_shard(xtr, ytr)
    eng.scoring = importance
    eng.prime()
    eng.step()
    eng.build_graphs()
    curve, t_train, reached = [], 0.0, None
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    for s in range(1, args.steps + 1):
        if s % args.eval_every == 1 or args.eval_every == 1:
            a.record()
        eng.step()
        if s % args.eval_every == 0:
            b.record()
            torch.cuda.synchronize()
            t_train += a.elapsed_time(b) / 1e3
            _, acc, _ = eng.evaluate_arrays(xte, yte)
            curve.append((s, round(t_train, 4), round(acc, 4)))
            if reached is None and acc >= args.target:
                reached = (s, t_train)
    return {'curve': curve, 'steps_to_target': reached[0] if reached else None,
            'seconds_to_target': round(reached[1], 3) if reached else None,
            'ms_per_step': round(1e3 * curve[-1][1] / curve[-1][0], 4) if curve else None,
            'final_acc': curve[-1][2] if curve else None}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=3000)
    ap.add_argument('--eval-every', type=int, default=100)
    ap.add_argument('--target', type=float, default=0.6)
    ap.add_argument('--model', default='resnet18')
    ap.add_argument('--lr', type=float, default=1e-3)
    ap.add_argument('--noise', type=int, default=64)
    ap.add_argument('--contrast', type=float, default=0.04)
    ap.add_argument('--hard-frac', type=float, default=0.1)
    ap.add_argument('--seed', type=int, default=3)
    args = ap.parse_args()
    x, y = make_data(12000, 10, 8, args.noise, args.hard_frac, args.contrast)
    xtr, ytr, xte, yte = x[:10000], y[:10000], x[10000:], y[10000:]
    out = {'bench': 'time_to_accuracy', 'model': args.model, 'target_acc': args.target,
           'data': 'synthetic cifar10-shape, template contrast %.2f, noise +-%d, %.0f%% '
                   'relabelled' % (args.contrast, args.noise, 100 * args.hard_frac)}
    t0 = time.time()
    out['importance'] = run(True, args, xtr, ytr, xte, yte)
    out['uniform'] = run(False, args, xtr, ytr, xte, yte)
    i, u = out['importance'], out['uniform']
    if i['seconds_to_target'] and u['seconds_to_target']:
        out['time_speedup_vs_uniform'] = round(u['seconds_to_target'] / i['seconds_to_target'], 3)
        out['step_speedup_vs_uniform'] = round(u['steps_to_target'] / i['steps_to_target'], 3)
    out['wall_s'] = round(time.time() - t0, 1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
