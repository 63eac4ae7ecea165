"""Where does a small (B=32) conv launch spend its ~12-20 us?  A/B in one process.

Variants of the same 1x1/s2 and 3x3 convs: with / without the BN-stats epilogue,
register-staged vs LDS-DMA main loop, plus floors: a trivial torch fill kernel and
a graph-replayed chain of 20 identical convs (per-kernel boundary cost).
"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan
    from conv_bench import timeit
    dev = 'cuda'
    small = torch.zeros(1024, device=dev)
    print('torch fill (floor)      %.1f us' % timeit(lambda: small.fill_(1.0), 100))
    for (C, K, H, R, st, pd) in [(64, 128, 32, 1, 2, 0), (64, 64, 32, 3, 1, 1),
                                 (512, 512, 4, 3, 1, 1)]:
        sp = ConvSpec(32, H, H, C, K, R, R, st, pd)
        x = ops.to_nhwc(torch.randn(32, C, H, H, device=dev))
        wk, _ = ops.pack_conv_weight(torch.randn(K, C, R, R, device=dev) * 0.05)
        y = torch.empty(sp.M, K, dtype=torch.bfloat16, device=dev)
        stats = torch.zeros(2, K, device=dev)
        plan = fwd_plan(sp)
        res = {}
        for name, kw in [('stats', dict(stats=stats)), ('nostats', {}),
                         ('nostats_nosplit', dict(plan=(64, 128 if K > 64 else 64, 1))),
                         ('pipe4', dict(stats=stats, pipe=4))]:
            kw.setdefault('plan', plan)
            res[name] = timeit(lambda: ops.conv_fwd(x, wk, y, sp, **kw), 100)
        # chain of 20 launches captured in a graph: per-launch cost in a dependent chain
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                ops.conv_fwd(x, wk, y, sp, plan=plan)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for _ in range(20):
                ops.conv_fwd(x, wk, y, sp, plan=plan)
        res['graph_chain_per_kernel'] = timeit(g.replay, 20) / 20
        print('C%d K%d H%d R%d s%d plan=%s: %s' % (C, K, H, R, st, plan, ', '.join(
            '%s=%.1fus' % kv for kv in res.items())), flush=True)


if __name__ == '__main__':
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
