"""Phase split of the halo conv (csrc/hconv.hip) from in-kernel s_memtime stamps.

Diagnostic build only: build with MERCURY_VARIANT_FLAGS=-DMERCURY_STAMPS python
bench/build_variant.py HEAD OUT.so, run with MERCURY_EXT_PATH=OUT.so.

    python bench/stamp_hconv.py N C K H stride [bm bn splits] [mode]
Prints median / p90 over blocks (shader clocks): prologue (entry -> first halo landed), main
loop, epilogue, and the main loop split summed over taps: wait+barrier, DMA issue, reads+MFMA,
slice starts (halo wait + transform).
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from mercury_amd import ops
    from mercury_amd.ops import hconv as H
    from mercury_amd.ops.conv import ConvSpec, slab_bytes
    a = [int(v) for v in sys.argv[1:]]
    N, C, K, Hh, st = a[:5]
    sp = ConvSpec(N, Hh, Hh, C, K, 3, 3, st, 1)
    if N > 32:
        sp.group_rows = 32 * sp.P * sp.Q
    plan = tuple(a[5:8]) if len(a) >= 8 else H.plan(sp)
    mode = a[8] if len(a) >= 9 else 0
    x = ops.to_nhwc(torch.randn(N, C, Hh, Hh, device='cuda'))
    wk, _ = ops.pack_conv_weight(torch.randn(K, C, 3, 3, device='cuda') * 0.05)
    y = torch.empty(sp.M, K, dtype=torch.bfloat16, device='cuda')
    G = N // 32 if N > 32 else 1
    stats = torch.zeros(G * 2 * K, device='cuda')
    slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4 + 1), device='cuda')
    pro = None
    if mode:
        pro = dict(stats=torch.rand(G * 2 * C, device='cuda') + 1, gamma=torch.ones(C, device='cuda'),
                   beta=torch.zeros(C, device='cuda'), act='relu', count=(32 if N > 32 else N) * Hh * Hh,
                   group_imgs=32 if N > 32 else N)
        if mode == 2:
            pro['res'] = x.clone()
    for _ in range(5):
        H.hconv_fwd(x, wk, y, sp, plan, stats=stats, slab=slab, pro=pro)
    torch.cuda.synchronize()
    ntiles = (sp.M // plan[0]) * ((K + plan[1] - 1) // plan[1])
    nb = min(ntiles, 256) if plan[2] == 0 else ntiles * plan[2]
    v = np.array(ops.lib().hconv_stamps(min(nb, 8192)), dtype=np.int64).reshape(-1, 12)
    if v.size == 0:
        print('not a stamps build')
        return
    if plan[2] == 0:
        # persistent kernel: prologue, loop, per-phase sums of wave 0 over all steps
        f = lambda q: '%8d %8d' % (np.median(q), np.percentile(q, 90))
        print('shape', a[:5], 'plan', plan, 'blocks', len(v), 'tiles/block %.2f' % (ntiles / len(v)))
        print('  prologue  med/p90 %s' % f(v[:, 1] - v[:, 0]))
        print('  loop      med/p90 %s' % f(v[:, 2] - v[:, 1]))
        names = ('mfma-half-1 issue', 'vmcnt wait', 'barrier', 'DMA issue', 'reads+mfma-half-2',
                 'epilogue')
        for q, nm in enumerate(names):
            print('  %-20s med/p90 %s' % (nm, f(v[:, 4 + q])))
        t0 = v[:, 0] - v[:, 0].min()
        print('  block start spread med/p90/max %d %d %d, kernel span %d' % (
            np.median(t0), np.percentile(t0, 90), t0.max(), v[:, 3].max() - v[:, 0].min()))
        return
    pro_, loop, epi = v[:, 1] - v[:, 0], v[:, 2] - v[:, 1], v[:, 3] - v[:, 2]
    t0 = v[:, 0] - v[:, 0].min()
    f = lambda q: '%7d %7d' % (np.median(q), np.percentile(q, 90))
    print('shape', a[:5], 'plan', plan, 'mode', mode, 'blocks', len(v))
    print('  prologue  med/p90 %s' % f(pro_))
    print('  mainloop  med/p90 %s' % f(loop))
    print('  epilogue  med/p90 %s' % f(epi))
    print('  loop split (median, summed over taps): wait+barrier %d  issue %d  reads+mfma %d  '
          'slice-start %d' % tuple(np.median(v[:, 4 + q]) for q in range(4)))
    e = lambda a_, b_: np.median(v[:, b_] - v[:, a_])
    print('  epilogue split (median): split-K/setup %d  acc->LDS tile + stats %d  '
          'sync + stats atomics %d  row stores %d' % (e(2, 8), e(8, 9), e(9, 10), e(10, 3)))
    print('  block start spread med/p90/max %d %d %d, kernel span %d' % (
        np.median(t0), np.percentile(t0, 90), t0.max(), v[:, 3].max() - v[:, 0].min()))


if __name__ == '__main__':
    main()
