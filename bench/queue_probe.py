"""Do two HIP streams share a hardware queue?  (Shared queue = serialised work.)

HIP maps every stream onto one of GPU_MAX_HW_QUEUES hardware queues per priority level; once
that many exist, a new stream shares the least-used one.  Two streams on one queue run their
work back to back, so the score / train / comm overlap of the engine's step silently turns
into serial execution (1.37 -> 2.1 ms/step in proxy_ab runs that built many engines in one
process).  This probe launches a one-block spin kernel (``torch.cuda._sleep``) on the default
stream and on each newly created stream at once and reports the wall time of the pair against
one spin alone: ~1x overlapped, ~2x shared.

    python bench/queue_probe.py [--streams 12] [--priorities 0,-1]
"""
import argparse
import json
import time

import torch


def pair_ms(s, cycles):
    d = torch.cuda.current_stream()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(cycles)
    with torch.cuda.stream(s):
        torch.cuda._sleep(cycles)
    torch.cuda.synchronize()
    del d
    return (time.perf_counter() - t0) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--streams', type=int, default=12)
    ap.add_argument('--priorities', default='0,-1')
    ap.add_argument('--cycles', type=int, default=20_000_000)
    ap.add_argument('--dist', action='store_true',
                    help='initialise a one-rank nccl (RCCL) process group first, as the DP path does')
    a = ap.parse_args()
    torch.cuda.init()
    if a.dist:
        import os
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from mercury_amd.parallel import dist as pdist
        pdist.init_from_env(force=True)
        import torch.distributed as tdist
        t = torch.ones(4, device='cuda')
        tdist.all_reduce(t)
        torch.cuda.synchronize()
    print('priority_range', torch.cuda.Stream.priority_range(), flush=True)
    torch.cuda._sleep(a.cycles)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    torch.cuda._sleep(a.cycles)
    torch.cuda.synchronize()
    one = (time.perf_counter() - t0) * 1e3
    res = {'one_spin_ms': round(one, 2)}
    for p in [int(x) for x in a.priorities.split(',')]:
        rows = []
        for i in range(a.streams):
            s = torch.cuda.Stream(priority=p)
            rows.append(round(pair_ms(s, a.cycles) / one, 2))
        res['priority_%d' % p] = rows
        print('priority %d: pair/one per new stream %s' % (p, rows), flush=True)
    # the engine's role streams (ops.role_stream: default-priority pool streams, cached)
    try:
        import os
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from mercury_amd import ops
        res['role_score'] = round(pair_ms(ops.role_stream('cuda:0', 'score'), a.cycles) / one, 2)
        res['role_comm'] = round(pair_ms(ops.role_stream('cuda:0', 'comm'), a.cycles) / one, 2)
        with torch.cuda.stream(ops.role_stream('cuda:0', 'score')):
            res['role_score_vs_comm'] = round(
                pair_ms(ops.role_stream('cuda:0', 'comm'), a.cycles) / one, 2)
    except ImportError as e:
        print('role streams unavailable:', e, flush=True)
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
