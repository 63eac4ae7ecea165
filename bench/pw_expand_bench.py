"""ResNet-50 B=1280 pointwise shapes: pgemm at each tile width vs pwconv (graph-timed, ghost-BN
statistics on), with an output and statistics cross-check of the two.

    python bench/pw_expand_bench.py
"""
import json, os, sys
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE)); sys.path.insert(0, os.path.join(os.path.dirname(HERE), 'bench'))
from gtime import gtime
import torch
from mercury_amd import ops
from mercury_amd.ops.conv import ConvSpec, pwconv_fwd, pgemm_fwd, pgemm_plan
ops.lib()
dev = 'cuda'
B, grp = 1280, 128
for (C, K, H) in [(64, 256, 56), (128, 512, 28), (64, 64, 56), (256, 1024, 14), (512, 2048, 7)]:
    sp = ConvSpec(B, H, H, C, K, 1, 1, 1, 0)
    sp.group_rows = grp * sp.P * sp.Q
    x = torch.randn(B * H * H * sp.Cp, device=dev).to(torch.bfloat16)
    w = (torch.randn(K * sp.Cp, device=dev) * 0.05).to(torch.bfloat16)
    y = torch.empty(sp.M * K, device=dev, dtype=torch.bfloat16)
    y2 = torch.empty(sp.M * K, device=dev, dtype=torch.bfloat16)
    stats = torch.zeros(10 * 2 * K, device=dev)
    stats2 = torch.zeros(10 * 2 * K, device=dev)
    row = {'shape': [C, K, H], 'plan': pgemm_plan(sp)}
    byt = (sp.N * H * H * C + sp.M * K) * 2
    for bn in (64, 128, 256):
        if bn > K: continue
        try:
            us = gtime(lambda bn=bn: pgemm_fwd(x, w, y, sp, stats=stats, bn=bn), reps=4, iters=5)
            row['pg%d' % bn] = [round(us, 1), round(byt / us / 1e3)]
        except Exception as e:
            row['pg%d' % bn] = str(e)[:60]
    if C <= 128:
        us = gtime(lambda: pwconv_fwd(x, w, y2, sp, stats=stats2), reps=4, iters=5)
        row['pw'] = [round(us, 1), round(byt / us / 1e3)]
        pgemm_fwd(x, w, y, sp, stats=stats.zero_(), bn=row['plan'] if isinstance(row['plan'], int) else 128)
        pwconv_fwd(x, w, y2, sp, stats=stats2.zero_())
        torch.cuda.synchronize()
        row['maxdiff_y'] = float((y.float() - y2.float()).abs().max())
        row['maxrel_stats'] = float(((stats - stats2).abs() / (stats2.abs() + 1e-3)).max())
    print(json.dumps(row), flush=True)
