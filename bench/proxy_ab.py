"""Upper bounds by omission: what the concurrent step would gain if a class of launches cost
nothing.  Each variant monkey-patches the engine BEFORE its graphs are captured (wrong numerics,
timing only -- never a result) and the variants are timed in interleaved rounds in ONE process
(cdna_hip_programming.md §5.4 rule 24).

    python bench/proxy_ab.py [--config resnet18-cifar10] [--rounds 3] [--steps 200]
        [--variants base,score_bn,train_fwd_bn,train_bwd_bn,all_bn]

Prints one JSON line: {variant: [ms/step per round]}.
"""
from __future__ import annotations
import os
if int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:   # before torch loads HIP: see
    os.environ['GPU_MAX_HW_QUEUES'] = '16'                # mercury_amd/__init__.py

import argparse
import json
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def patches(name):
    """{method: replacement factory} of a variant (applied to one engine instance)."""
    def skip_bn_apply(which):
        def wrap(eng):
            orig = eng._bn_apply

            def f(m, *a, **k):
                if which(m):
                    return None
                return orig(m, *a, **k)
            eng._bn_apply = f
        return wrap

    def skip_bn_bwd(eng):
        eng._bn_bwd = lambda *a, **k: None

    def skip_comm(eng):
        # DP machinery kept (segmented graphs, comm-stream event edges), collective skipped
        class NoComm(object):
            size = eng.comm.size

            def allreduce(self, t, avg=True):
                return t
        eng.comm = NoComm()

    table = {
        'base': [],
        'score_bn': [skip_bn_apply(lambda m: not m.train)],
        'train_fwd_bn': [skip_bn_apply(lambda m: m.train)],
        'train_bwd_bn': [skip_bn_bwd],
        'all_bn': [skip_bn_apply(lambda m: True), skip_bn_bwd],
        'dp': [],                      # (--dp: every variant runs forced buckets)
        'dp_nocomm': [skip_comm],
    }
    return table[name]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='resnet18-cifar10')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--variants', default='base,score_bn,train_fwd_bn,train_bwd_bn,all_bn')
    ap.add_argument('--dp', default='',
                    help="comma list of variants run with forced DP buckets (RCCL, W = 1)")
    ap.add_argument('--opts', default='',
                    help="'|'-separated EngineOptions specs, one per variant named opt<i>")
    args = ap.parse_args()
    import numpy as np
    import torch
    import bench as B
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model

    pre = B.PRESETS[args.config]
    hw, x_all, y_all = B.preset_data(pre)
    dev = torch.device('cuda:0')
    torch.manual_seed(1234)
    net = build_model(pre['model'], pre['classes']).to(dev)
    res = {}
    names = args.variants.split(',')
    dp = set(filter(None, args.dp.split(',')))
    optspecs = [o for o in args.opts.split('|') if o] if args.opts else []
    names += ['opt%d' % i for i in range(len(optspecs))]
    if dp:
        from mercury_amd.parallel import dist as pdist
        pdist.init_from_env(force=True)
    from mercury_amd.config import EngineOptions
    for rnd in range(args.rounds):
        for name in names:
            opts = None
            if name.startswith('opt'):
                os.environ['MERCURY_ENGINE_OPTS'] = optspecs[int(name[3:])]
                opts = EngineOptions.from_env()
                os.environ.pop('MERCURY_ENGINE_OPTS')
            eng = NativeEngine(net, dev, pre['batch'], 10, optimizer='adam', lr=0.001, seed=7,
                               image_hw=hw, force_buckets=name in dp, opts=opts)
            for p in patches(name) if not name.startswith('opt') else []:
                p(eng)
            eng.set_shard(x_all, y_all)
            eng.prime()
            eng.step()
            eng.build_graphs()
            for _ in range(args.warmup):
                eng.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                eng.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            res.setdefault(name, []).append(round(ms, 4))
            print('[proxy] round %d %-14s %.4f ms/step' % (rnd, name, ms), flush=True)
            del eng
            torch.cuda.synchronize()
    print(json.dumps({'config': args.config, 'ms_per_step': res,
                      'note': 'omission upper bounds: wrong numerics, timing only'}), flush=True)


if __name__ == '__main__':
    main()
