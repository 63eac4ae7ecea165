"""Time-to-accuracy: importance sampling vs uniform sampling (Mercury's actual claim).

Mercury trades per-step throughput (every step also scores a 10x32 pool) for
fewer steps to a target accuracy.  For each of ``--seeds`` seeds (model init,
sampling and augmentation streams) this runs the native engine twice on the
same synthetic CIFAR-10-shaped shard -- once with the reference importance
sampler (`pytorch_collab.py:108-116`), once uniform -- evaluates held-out
accuracy every ``--eval-every`` steps on ``--test`` held-out samples, and
reports, per seed and as mean +- std over seeds: accuracy at every checkpoint,
steps and wall time (event-timed train steps only, evaluation excluded) to
reach ``--target``, and the IS-minus-uniform accuracy gap in units of its
standard error at the first checkpoint where the IS mean reaches the target.

The synthetic task (low-contrast class templates under pixel noise, plus a fraction of
relabelled "hard" samples) is NOT CIFAR-10, so the numbers measure the
mechanism, not the paper's accuracy curve (no dataset download is possible).

    python bench/time_to_accuracy.py [--steps 3000] [--seeds 5] [--target 0.6] > tta.json
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


def run(importance, args, seed, xtr, ytr, xte, yte):
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    torch.manual_seed(seed)
    net = build_model(args.model, 10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, lr=args.lr, seed=11 + 7 * seed, importance=importance,
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
    eng.close()
    return {'curve': curve, 'steps_to_target': reached[0] if reached else None,
            'seconds_to_target': round(reached[1], 3) if reached else None,
            'ms_per_step': round(1e3 * curve[-1][1] / curve[-1][0], 4) if curve else None,
            'final_acc': curve[-1][2] if curve else None}


def summarise(runs, target):
    """mean / std over seeds of accuracy at each checkpoint, steps to target."""
    steps = [c[0] for c in runs[0]['curve']]
    accs = np.array([[c[2] for c in r['curve']] for r in runs])
    reach = [r['steps_to_target'] for r in runs]
    hit = [x for x in reach if x is not None]
    return {'steps': steps, 'acc_mean': [round(float(v), 4) for v in accs.mean(0)],
            'acc_std': [round(float(v), 4) for v in accs.std(0, ddof=1)] if len(runs) > 1
            else None,
            'steps_to_target_per_seed': reach,
            'seeds_reaching_target': '%d/%d' % (len(hit), len(runs)),
            'steps_to_target_mean': round(float(np.mean(hit)), 1) if hit else None,
            'steps_to_target_std': round(float(np.std(hit, ddof=1)), 1) if len(hit) > 1 else None}


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
    ap.add_argument('--seeds', type=int, default=5)
    ap.add_argument('--seed0', type=int, default=3)
    ap.add_argument('--train', type=int, default=10000)
    ap.add_argument('--test', type=int, default=6000)
    args = ap.parse_args()
    x, y = make_data(args.train + args.test, 10, 8, args.noise, args.hard_frac, args.contrast)
    xtr, ytr = x[:args.train], y[:args.train]
    xte, yte = x[args.train:], y[args.train:]
    out = {'bench': 'time_to_accuracy', 'model': args.model, 'target_acc': args.target,
           'seeds': [args.seed0 + k for k in range(args.seeds)], 'held_out': args.test,
           'data': 'synthetic cifar10-shape, template contrast %.2f, noise +-%d, %.0f%% '
                   'relabelled' % (args.contrast, args.noise, 100 * args.hard_frac)}
    t0 = time.time()
    per = {'importance': [], 'uniform': []}
    for k in range(args.seeds):
        seed = args.seed0 + k
        for name, imp in (('importance', True), ('uniform', False)):
            r = run(imp, args, seed, xtr, ytr, xte, yte)
            r['seed'] = seed
            per[name].append(r)
            print('[tta] seed %d %s: steps to %.2f = %s, final acc %.4f' % (
                seed, name, args.target, r['steps_to_target'], r['final_acc']),
                file=sys.stderr, flush=True)
    out['per_seed'] = per
    out['importance'] = summarise(per['importance'], args.target)
    out['uniform'] = summarise(per['uniform'], args.target)
    i, u = out['importance'], out['uniform']
    # the IS - uniform gap at the first checkpoint where the IS mean reaches the target, in
    # units of the standard error of the difference of the two seed means
    n = args.seeds
    for j, st in enumerate(i['steps']):
        if i['acc_mean'][j] >= args.target:
            gap = i['acc_mean'][j] - u['acc_mean'][j]
            se = ((i['acc_std'][j] ** 2 + u['acc_std'][j] ** 2) / n) ** 0.5 if n > 1 else None
            out['at_target_step'] = {'step': st, 'is_acc_mean': i['acc_mean'][j],
                                     'uniform_acc_mean': u['acc_mean'][j], 'gap': round(gap, 4),
                                     'gap_in_std_err': round(gap / se, 2) if se else None,
                                     'is_acc_std': i['acc_std'][j] if n > 1 else None,
                                     'uniform_acc_std': u['acc_std'][j] if n > 1 else None}
            break
    ti = [r['seconds_to_target'] for r in per['importance']]
    if all(ti):
        out['is_seconds_to_target_mean'] = round(float(np.mean(ti)), 3)
    out['wall_s'] = round(time.time() - t0, 1)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
