"""Does the native engine LEARN on a preset's architecture and input shape?

    python bench/learn_check.py --config resnet50-imagenet --classes 10 --steps 300

Trains the preset's model (random init, the preset's per-GPU batch and 10x scoring pool,
importance sampling on) on a learnable class-conditional synthetic set
(data.datasets.synthetic_arrays: low-frequency class templates + noise) and prints one JSON
line: the train-loss curve (mean weighted CE per 25-step window, from the device meters),
held-out loss / accuracy before and after (running-stat BN), and ms per step.  The headline
bench uses the preset's full class count, where a few hundred steps cannot show learning.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='resnet50-imagenet')
    ap.add_argument('--classes', type=int, default=10)
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--n', type=int, default=6400)
    ap.add_argument('--lr', type=float, default=1e-3)
    args = ap.parse_args()
    import torch
    import bench as B
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    pre = B.PRESETS[args.config]
    hw = pre['hw'] if isinstance(pre['hw'], tuple) else (pre['hw'], pre['hw'])
    x, y = synthetic_arrays(args.n, args.classes, shape=(hw[0], hw[1], 3), seed=8)
    xt, yt = synthetic_arrays(1000, args.classes, shape=(hw[0], hw[1], 3), seed=9)
    torch.manual_seed(1234)
    net = build_model(pre['model'], args.classes).cuda()
    eng = NativeEngine(net, 'cuda', pre['batch'], 10, optimizer='adam', lr=args.lr, seed=7,
                       image_hw=hw)
    eng.set_shard(x, y)
    l0, a0, _ = eng.evaluate_arrays(xt, yt, batch=250)
    eng.prime()
    eng.step()
    eng.build_graphs()
    curve, win = [], 25
    t0 = time.perf_counter()
    done = 1
    while done < args.steps:
        eng.meters[:3].zero_()
        for _ in range(min(win, args.steps - done)):
            eng.step()
            done += 1
        m = eng.read_meters()
        curve.append(round(m['loss_sum'] / max(m['count'], 1), 4))
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1e3 / (args.steps - 1)
    l1, a1, _ = eng.evaluate_arrays(xt, yt, batch=250)
    out = dict(config=args.config, model=pre['model'], image_hw=list(hw), classes=args.classes,
               per_gpu_batch=pre['batch'], presample_pool=pre['batch'] * 10, steps=args.steps,
               train_loss_windows=curve, initial_window_loss=curve[0], final_window_loss=curve[-1],
               chance_loss=round(math.log(args.classes), 4),
               heldout_before=dict(loss=round(l0, 4), acc=round(a0, 4)),
               heldout_after=dict(loss=round(l1, 4), acc=round(a1, 4)),
               ms_per_step_incl_window_reads=round(ms, 2), data='synthetic class templates + noise')
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
