"""Does initialising torch.distributed (RCCL) slow an engine step down in the same process?

Times the ResNet-18 preset step of one engine built BEFORE the process group exists, then
initialises a one-rank nccl (RCCL) group, times the same engine again, builds a second engine
and times it.  For each it reports device ms/step (synchronised wall over the loop) and the
host time per ``step()`` call (no sync), which separates a host-bound step from a GPU one.

    python bench/dist_probe.py [--steps 200]
"""
import os
if int(os.environ.get('GPU_MAX_HW_QUEUES') or 0) < 16:   # before torch loads HIP: see
    os.environ['GPU_MAX_HW_QUEUES'] = '16'                # mercury_amd/__init__.py
import argparse
import json
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_engine(eng, steps, torch):
    for _ in range(20):
        eng.step()
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for _ in range(steps):
        h0 = time.perf_counter()
        eng.step()
        host += time.perf_counter() - h0
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / steps
    return round(wall, 4), round(host * 1e3 / steps, 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=200)
    ap.add_argument('--dist-first', action='store_true',
                    help='initialise the process group before building any engine (DP order)')
    a = ap.parse_args()
    import torch
    import bench as B
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    from mercury_amd.parallel import dist as pdist
    pre = B.PRESETS['resnet18-cifar10']
    hw, x_all, y_all = B.preset_data(pre)
    dev = torch.device('cuda:0')
    torch.manual_seed(1234)
    net = build_model(pre['model'], pre['classes']).to(dev)

    def make(**kw):
        eng = NativeEngine(net, dev, pre['batch'], 10, optimizer='adam', lr=0.001, seed=7,
                           image_hw=hw, **kw)
        eng.set_shard(x_all, y_all)
        eng.prime()
        eng.step()
        eng.build_graphs()
        return eng

    res = {}
    if a.dist_first:
        pdist.init_from_env(force=True)
    e1 = make()
    res['engine1_before_dist' if not a.dist_first else 'engine1_dist_first'] = \
        time_engine(e1, a.steps, torch)
    if not a.dist_first:
        pdist.init_from_env(force=True)
        res['engine1_after_dist'] = time_engine(e1, a.steps, torch)
    e2 = make()
    res['engine2_after_dist'] = time_engine(e2, a.steps, torch)
    e3 = make(force_buckets=True)
    res['engine3_forced_buckets'] = time_engine(e3, a.steps, torch)
    res['engine1_again'] = time_engine(e1, a.steps, torch)
    print(json.dumps({'ms_per_step_and_host_ms_per_call': res}), flush=True)


if __name__ == '__main__':
    main()
