"""Where does a conv block spend its time?  Phase split of the register-staged igemm body from
in-kernel s_memtime stamps (diagnostic build: bench/build_variant.py-style build with
-DMERCURY_STAMPS, loaded through MERCURY_EXT_PATH).

    python bench/stamp_conv.py N C K H R stride pad
Prints median / p90 over blocks (shader clocks) of: prologue (entry -> first stage staged),
main loop, epilogue, plus the spread of block start times.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    from mercury_amd import ops
    from mercury_amd.ops.conv import ConvSpec, fwd_plan, slab_bytes
    N, C, K, H, R, st, pd = (int(v) for v in sys.argv[1:8])
    sp = ConvSpec(N, H, H, C, K, R, R, st, pd)
    if N > 32:
        sp.group_rows = 32 * sp.P * sp.Q
    x = ops.to_nhwc(torch.randn(N, C, H, H, device='cuda'))
    wk, _ = ops.pack_conv_weight(torch.randn(K, C, R, R, device='cuda') * 0.05)
    y = torch.empty(sp.M, K, dtype=torch.bfloat16, device='cuda')
    G = N // 32 if N > 32 else 1
    stats = torch.zeros(G * 2 * K, device='cuda')
    plan = fwd_plan(sp)
    slab = torch.zeros(max(1, slab_bytes(sp.M, K, *plan) // 4), device='cuda')
    for _ in range(5):
        ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab, plan=plan)
    torch.cuda.synchronize()
    ops.conv_fwd(x, wk, y, sp, stats=stats, slab=slab, plan=plan)
    torch.cuda.synchronize()
    nb = (sp.M + plan[0] - 1) // plan[0] * ((K + plan[1] - 1) // plan[1]) * plan[2]
    v = np.array(ops.lib().igemm_stamps(min(nb, 8192)), dtype=np.int64).reshape(-1, 12)
    if v.size == 0:
        print('not a stamps build')
        return
    pro, loop, epi = v[:, 1] - v[:, 0], v[:, 2] - v[:, 1], v[:, 3] - v[:, 2]
    t0 = v[:, 0] - v[:, 0].min()
    f = lambda a: '%7d %7d' % (np.median(a), np.percentile(a, 90))
    print('shape', sys.argv[1:8], 'plan', plan, 'blocks', len(v))
    print('  prologue  med/p90 %s' % f(pro))
    print('  mainloop  med/p90 %s' % f(loop))
    print('  epilogue  med/p90 %s' % f(epi))
    print('  main-loop split (median cycles summed over stages): load-issue %d  mfma %d  '
          'store(+load wait) %d  barrier %d' % tuple(np.median(v[:, 4 + q]) for q in range(4)))
    e = lambda a, b: np.median(v[:, b] - v[:, a])
    print('  epilogue split (median): split-K/setup %d  acc->LDS tile + stats %d  '
          'sync + stats atomics %d  row stores %d' % (e(2, 8), e(8, 9), e(9, 10), e(10, 3)))
    print('  block start spread med/p90/max %d %d %d, kernel span %d' % (
        np.median(t0), np.percentile(t0, 90), t0.max(), v[:, 3].max() - v[:, 0].min()))


if __name__ == '__main__':
    main()
