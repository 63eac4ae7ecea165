"""Host-vs-device time of the native step: is the step launch-bound?

Times N steps three ways: host wall time of the issuing loop (no sync), device
time of the whole loop (events), and per-graph replay cost, for graph and eager
mode.  Used to decide how much of the step is host submission.
"""
from __future__ import annotations

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    x, y = synthetic_arrays(20000, 10, seed=8)
    for graphs, fork in ((True, False), (True, True), (False, False), (False, True)):
        torch.manual_seed(0)
        net = ResNet18(10).cuda()
        eng = NativeEngine(net, 'cuda', 32, 10, use_graphs=graphs)
        if not fork:
            eng.s_wgrad = None
        print('--- fork_wgrad=%s' % fork)
        eng.set_shard(x, y)
        eng.prime()
        eng.step()
        if graphs:
            eng.build_graphs()
        for _ in range(10):
            eng.step()
        torch.cuda.synchronize()
        n = 50
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        t0 = time.perf_counter()
        for _ in range(n):
            eng.step()
        th = time.perf_counter() - t0
        e1.record()
        torch.cuda.synchronize()
        tt = time.perf_counter() - t0
        print('graphs=%s host_issue=%.3f ms/step wall=%.3f ms/step device=%.3f ms/step' % (
            graphs, th * 1e3 / n, tt * 1e3 / n, e0.elapsed_time(e1) / n), flush=True)
        if graphs:
            for name in ('score', 'tail'):
                g = eng.graphs[name]
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(20):
                    g.replay()
                th = time.perf_counter() - t0
                torch.cuda.synchronize()
                tt = time.perf_counter() - t0
                print('  replay %s: host %.1f us, wall %.1f us' % (name, th * 1e6 / 20, tt * 1e6 / 20))
            g = eng.graphs['train'][0][0]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                g.replay()
            th = time.perf_counter() - t0
            torch.cuda.synchronize()
            tt = time.perf_counter() - t0
            print('  replay train: host %.1f us, wall %.1f us' % (th * 1e6 / 20, tt * 1e6 / 20))
        del eng


if __name__ == '__main__':
    main()
