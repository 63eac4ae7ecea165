"""Tune the conv plans of bench.py's flagship step in situ (mercury_amd/ops/step_tune.py) and
write the result as a tune cache.

    python bench/step_tune.py --out gpurun_out/step_tune.json [--budget 600]
    MERCURY_TUNE_CACHE=gpurun_out/step_tune.json python bench.py     # use it
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--out', required=True)
    ap.add_argument('--budget', type=float, default=600.0)
    ap.add_argument('--steps', type=int, default=40)
    ap.add_argument('--chunks', type=int, default=3)
    ap.add_argument('--threshold', type=float, default=0.004)
    ap.add_argument('--config', default='resnet18-cifar10')
    ap.add_argument('--kinds', default='fwd,bwd', help="coordinates to tune: 'fwd', 'bwd'")
    args = ap.parse_args()
    os.environ['MERCURY_TUNE_CACHE'] = os.path.abspath(args.out) + '.none'   # start untuned
    import torch
    from bench import PRESETS, preset_data
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    from mercury_amd.ops import step_tune
    pre = PRESETS[args.config]
    hw, x, y = preset_data(pre)
    torch.manual_seed(1234)
    net = build_model(pre['model'], pre['classes']).cuda()
    eng = NativeEngine(net, 'cuda', pre['batch'], 10, optimizer='adam', lr=0.001, seed=7,
                       importance=True, world_size=1, use_graphs=True, image_hw=hw)
    eng.set_shard(x, y)
    eng.prime()
    eng.step()
    eng.build_graphs()
    for _ in range(30):
        eng.step()
    res, base, final = step_tune.tune_step(eng, steps=args.steps, chunks=args.chunks,
                                           threshold=args.threshold, budget_s=args.budget,
                                           kinds=tuple(args.kinds.split(',')),
                                           log=lambda s: print(s, flush=True))
    with open(args.out, 'w') as f:
        json.dump(dict(sorted(res.items())), f, indent=0, sort_keys=True)
    print(json.dumps({'baseline_ms': round(base, 4), 'tuned_ms': round(final, 4),
                      'coordinates': len(res), 'out': args.out}), flush=True)


if __name__ == '__main__':
    main()
