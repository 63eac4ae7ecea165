"""When does each stream of the native step actually run?  (no profiler attached)

Replays the step's graphs by hand with events around each replay and reports, per step,
the event times relative to the step start: score graph start/end (score stream), train
graph start/end (main stream), tail.  Two submission orders: score graph first (the
engine's order) and train graph first.

    python bench/stream_probe.py
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mercury_amd.data.datasets import synthetic_arrays
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import ResNet18
    x, y = synthetic_arrays(20000, 10, seed=8)
    torch.manual_seed(0)
    net = ResNet18(10).cuda()
    eng = NativeEngine(net, 'cuda', 32, 10, use_graphs=True)
    eng.set_shard(x, y)
    eng.prime()
    eng.step()
    eng.build_graphs()
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    s0 = torch.cuda.current_stream()
    ss = eng.s_score
    G = eng.graphs

    def ev():
        return torch.cuda.Event(enable_timing=True)

    for order in ('score_first', 'train_first', 'score_first'):
        acc = None
        n = 30
        for it in range(n + 5):
            e = {k: ev() for k in ('start', 'sc0', 'sc1', 'tr0', 'tr1', 'end')}
            e['start'].record(s0)
            ss.wait_event(e['start'])

            def score():
                with torch.cuda.stream(ss):
                    e['sc0'].record(ss)
                    G['score'].replay()
                    e['sc1'].record(ss)

            def train():
                e['tr0'].record(s0)
                for g, _, _ in G['train']:
                    g.replay()
                e['tr1'].record(s0)
            if order == 'score_first':
                score()
                train()
            else:
                train()
                score()
            s0.wait_event(e['sc1'])
            G['tail'].replay()
            e['end'].record(s0)
            torch.cuda.synchronize()
            if it < 5:
                continue
            v = {k: e['start'].elapsed_time(e[k]) * 1e3 for k in e if k != 'start'}
            acc = v if acc is None else {k: acc[k] + v[k] for k in v}
        print(order, ' '.join('%s=%.1f' % (k, acc[k] / n) for k in acc), flush=True)


if __name__ == '__main__':
    main()
