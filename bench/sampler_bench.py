"""Microbenchmark of the importance-sampling kernels (event-timed, graph-free).

    python bench/sampler_bench.py            -> JSON lines

* ``is_sample`` (pool sampler: EMA replay + probabilities + B draws), alias-table vs
  inverse-CDF draw, at pool sizes 320 (reference), 1280, 10240;
* ``ImportanceTable.sample`` (global HBM table: segment partials + fp64 scan + draws) at
  50k (CIFAR) and 1.28M (ImageNet) entries, 32 and 4096 draws.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, iters=200, warm=20):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    from mercury_amd import ops
    dev = 'cuda'
    for P in (320, 1280, 10240):
        B = 32
        losses = torch.rand(P, device=dev) * 3
        ema = torch.zeros(2, device=dev)
        ctrl = torch.zeros(8, dtype=torch.int64, device=dev)
        idx = torch.empty(B, dtype=torch.int32, device=dev)
        w = torch.empty(B, device=dev)
        for alias in (True, False):
            us = timed(lambda: ops.is_sample(losses, ema, ctrl, idx, w, P, B, 32, alias=alias))
            print(json.dumps({'kernel': 'is_sample', 'pool': P, 'draws': B,
                              'mode': 'alias' if alias else 'cdf', 'us': round(us, 2)}))
    for N in (50000, 1281167):
        t = ops.ImportanceTable(N, dev)
        t.write(0, torch.rand(N, device=dev), 1)
        for nd in (32, 4096):
            out = torch.empty(nd, dtype=torch.int64, device=dev)
            us = timed(lambda: t.sample(nd, 1, seed=3, out=out))
            print(json.dumps({'kernel': 'table_sample', 'table': N, 'draws': nd, 'us': round(us, 2)}))


if __name__ == '__main__':
    main()
