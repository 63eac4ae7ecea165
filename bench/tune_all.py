"""Autotune every conv plan used by the bench configs and write the cache.

    MERCURY_TUNE_CACHE=out.json python bench/tune_all.py [config ...]

Builds the native engine for each ``bench.py`` preset (train batch + scoring pool) with
autotuning on, which times every candidate plan for every conv shape (ops/tune.py) and stores
the winners; the resulting JSON is shipped as ``mercury_amd/ops/tune_cache.json``.
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from mercury_amd.engine.native import NativeEngine
    from mercury_amd.models import build_model
    from mercury_amd.ops import tune
    tune.enable(True)
    names = sys.argv[1:] or list(bench.PRESETS)
    for name in names:
        pre = bench.PRESETS[name]
        hw = pre['hw'] if isinstance(pre['hw'], tuple) else (pre['hw'], pre['hw'])
        t0 = time.time()
        net = build_model(pre['model'], pre['classes']).cuda()
        eng = NativeEngine(net, 'cuda', pre['batch'], 10, image_hw=hw, use_graphs=False)
        n = max(4 * pre['batch'], 64)
        if pre.get('chans', 3) == 3:
            x = np.random.randint(0, 255, (n, hw[0], hw[1], 3), dtype=np.uint8)
        else:
            x = np.random.randn(n, pre['chans'], hw[0], hw[1]).astype(np.float32)
        eng.set_shard(x, np.random.randint(0, pre['classes'], n))
        print('[tune] %s: %d cached plans, %.1f s' % (name, len(tune.cache()), time.time() - t0),
              flush=True)
        tune.save()
        del eng, net
        torch.cuda.empty_cache()


if __name__ == '__main__':
    main()
