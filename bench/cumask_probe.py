"""Spatial partitioning probe: the headline step with the scoring and train streams on
CU-masked HIP queues (hipExtStreamCreateWithCUMask) instead of sharing every CU.

    python bench/cumask_probe.py --split none|all|alt|half|xcd [--score-cus 128] [--steps 300]

``none``: the engine's ordinary streams (baseline).  ``all``: both streams CU-masked to every CU
(isolates the cost of a masked queue).  ``alt``: scoring on even CUs, training on odd ones;
``half``: scoring on CUs [0, S), training on the rest; ``xcd``: the split by hardware id modulo 8
(whichever CU numbering the mask uses, one of alt / half keeps XCDs whole).  The parent imports
nothing from torch before the engine; prints one JSON line.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _hip():
    for ln in open('/proc/self/maps'):
        if 'libamdhip64.so' in ln:
            return ctypes.CDLL(ln.split()[-1])
    return ctypes.CDLL('libamdhip64.so')


def masked_stream(torch, cus, mask_bits):
    hip = _hip()
    words = (cus + 31) // 32
    arr = (ctypes.c_uint32 * words)()
    for c in mask_bits:
        arr[c // 32] |= 1 << (c % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), arr)
    if rc != 0:
        raise RuntimeError('hipExtStreamCreateWithCUMask failed: %d' % rc)
    return torch.cuda.ExternalStream(s.value)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--split', default='none', choices=('none', 'all', 'alt', 'half', 'xcd'))
    ap.add_argument('--score-cus', type=int, default=0, help='CUs of the scoring stream (0: half)')
    ap.add_argument('--steps', type=int, default=300)
    ap.add_argument('--warmup', type=int, default=30)
    ap.add_argument('--train-prio', type=int, default=0,
                    help='priority of the train stream (-1: high; 0: the default stream)')
    args = ap.parse_args()
    import numpy as np
    import torch
    from mercury_amd import ops
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    from bench import PRESETS, preset_data

    dev = torch.device('cuda', 0)
    torch.cuda.init()
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    S = args.score_cus or cus // 2
    train_s = None
    if args.split != 'none':
        allc = list(range(cus))
        # scoring takes the first S CUs of the split's order, training the rest
        key = {'alt': lambda c: (c % 2, c), 'half': lambda c: c,
               'xcd': lambda c: (c % 8 >= 4, c)}
        if args.split == 'all':
            sc, tr = allc, allc
        else:
            order = sorted(allc, key=key[args.split])
            sc, tr = order[:S], order[S:]
        ops._ROLE_STREAMS[(0, 0)] = {'score': masked_stream(torch, cus, sc),
                                     'comm': torch.cuda.Stream(dev)}
        train_s = masked_stream(torch, cus, tr)
    if args.train_prio and train_s is None:
        train_s = torch.cuda.Stream(dev, priority=args.train_prio)
    pre = PRESETS['resnet18-cifar10']
    hw, x_all, y_all = preset_data(pre)
    torch.manual_seed(1234)
    net = build_model(pre['model'], pre['classes']).to(dev)
    eng = NativeEngine(net, dev, pre['batch'], 10, optimizer='adam', lr=0.001, seed=7,
                       importance=True, use_graphs=True, image_hw=hw)
    eng.set_shard(x_all, y_all)
    ctx = torch.cuda.stream(train_s) if train_s is not None else torch.cuda.stream(
        torch.cuda.current_stream(dev))
    with ctx:
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
        dt = (time.perf_counter() - t0) * 1e3 / args.steps
    eng.close()
    print(json.dumps({'split': args.split, 'train_prio': args.train_prio,
                      'score_cus': S if args.split != 'none' else None,
                      'cus': cus, 'ms_per_step': round(dt, 4)}), flush=True)


if __name__ == '__main__':
    main()
