"""Device time of a short launch sequence, measured by HIP-graph replay.

Timing small kernels with an event pair around each eager call measures the HOST: a
Python op call + pybind + hipLaunchKernel costs ~10-15 us, so every kernel shorter than
that reads as the host issue interval (the earlier per-layer sweeps at batch 32 did
exactly that).  Here ``fn`` is captured ``reps`` times into one graph and the replay is
event-timed, so the result is the in-graph cost per call -- kernel time plus the
dependent-boundary cost the real step pays (MI355X_MICROARCH.md, row 'boundary').

    from gtime import gtime
    us = gtime(lambda: ops.conv_fwd(...), reps=16)
"""
from __future__ import annotations


def gtime(fn, reps=16, iters=7):
    """Median microseconds per ``fn()`` over ``iters`` replays of a ``reps``-call graph.
    ``fn`` must only launch kernels on the current stream (no allocation, no sync)."""
    import torch
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.graph(g, stream=s, capture_error_mode='thread_local'):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(iters):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3 / reps)
    ts.sort()
    del g
    return ts[len(ts) // 2]
