"""Classifier-head kernels, graph-timed: forward (pool + FC + log-softmax CE, score and train
modes) and backward at the presets' head shapes.  The head path is read once per process
(MERCURY_HEAD_PATH: 0 auto, 1 per-sample kernel, 2 pool + split GEMM), so run one process per
setting.

    MERCURY_HEAD_PATH=2 python bench/head_bench.py
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from gtime import gtime  # noqa: E402

# (name, B, HW, C, classes)
SHAPES = [('mobilenetv2', 320, 16, 1280, 100), ('mobilenetv2', 32, 16, 1280, 100),
          ('resnet18', 320, 16, 512, 10), ('resnet18', 32, 16, 512, 10),
          ('resnet50', 1280, 49, 2048, 1000), ('resnet50', 128, 49, 2048, 1000)]


def main():
    import torch
    from mercury_amd import ops
    ops.lib()
    dev = 'cuda'
    for name, B, HW, C, K in SHAPES:
        act = torch.randn(B * HW * C, device=dev).to(torch.bfloat16)
        w = torch.randn(K * C, device=dev) * 0.02
        b = torch.zeros(K, device=dev)
        label = torch.randint(0, K, (B,), device=dev, dtype=torch.int32)
        pooled = torch.zeros(B, C, device=dev)
        logits = torch.zeros(B, K, device=dev)
        dlogits = torch.zeros(B, K, device=dev)
        losses = torch.zeros(B, device=dev)
        isw = torch.ones(B, device=dev)
        meters = torch.zeros(8, device=dev)
        dw = torch.zeros(K * C, device=dev)
        db = torch.zeros(K, device=dev)
        dact = torch.empty(B * HW * C, device=dev, dtype=torch.bfloat16)
        mode = 'score' if B in (320, 1280) else 'train'

        def fwd():
            ops.head_fwd(act, w, b, label, B, HW, C, K, mode, pooled=pooled, logits=logits,
                         dlogits=dlogits if mode == 'train' else None, losses=losses,
                         isw=isw if mode == 'train' else None, meters=meters)
        t_f = gtime(fwd, reps=8)
        rec = dict(net=name, B=B, HW=HW, C=C, classes=K, mode=mode, fwd_us=round(t_f, 1),
                   path=os.environ.get('MERCURY_HEAD_PATH', '0'))
        if mode == 'train':
            t_b = gtime(lambda: ops.head_bwd(pooled, dlogits, w, dw, db, dact, B, HW, C, K),
                        reps=8)
            rec['bwd_us'] = round(t_b, 1)
        print(json.dumps(rec), flush=True)


if __name__ == '__main__':
    main()
