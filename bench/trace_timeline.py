"""Per-queue timeline summary of a rocprofv3 ``--kernel-trace`` capture.

    python bench/trace_timeline.py <rocprof out dir> [last_n_steps_marker_kernel] [n_steps]

Reports, over the trailing window that contains the last ``n_steps`` launches of
the marker kernel (default ``optimizer_kernel``, once per step): wall time per
step, per-queue kernel count / busy time / idle gaps, and the launch-floor share
(kernels shorter than 8 us).  Used to decide whether a stream is kernel-bound or
gap (launch) bound.
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'optimizer_kernel'
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    f = glob.glob(root + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        r['s'] = int(r['Start_Timestamp'])
        r['e'] = int(r['End_Timestamp'])
    rows.sort(key=lambda r: r['s'])
    marks = [r for r in rows if marker in r['Kernel_Name']]
    if len(marks) < nsteps + 1:
        nsteps = len(marks) - 1
    t0, t1 = marks[-nsteps - 1]['e'], marks[-1]['e']
    win = [r for r in rows if r['s'] >= t0 and r['e'] <= t1]
    qkey = 'Queue_Id' if 'Queue_Id' in rows[0] else 'Stream_Id'
    byq = defaultdict(list)
    for r in win:
        byq[r[qkey]].append(r)
    wall = (t1 - t0) / 1e3 / nsteps
    print('window: %d steps, wall %.1f us/step, %d kernels/step' % (nsteps, wall, len(win) / nsteps))
    for q, ks in sorted(byq.items()):
        busy = sum(k['e'] - k['s'] for k in ks) / 1e3 / nsteps
        small = sum(1 for k in ks if k['e'] - k['s'] < 8000) / nsteps
        gaps = []
        for a, b in zip(ks, ks[1:]):
            gaps.append(max(0, b['s'] - a['e']))
        g = sorted(gaps)
        med = g[len(g) // 2] / 1e3 if g else 0
        print('queue %s: %5.1f kernels/step, busy %7.1f us/step (%4.1f%% of wall), '
              'median gap %.1f us, %4.1f kernels/step < 8us'
              % (q, len(ks) / nsteps, busy, 100 * busy / wall, med, small))
    # union of busy intervals: how much of the wall has no kernel running at all
    iv = sorted((r['s'], r['e']) for r in win)
    union, cs, ce = 0, None, None
    for s_, e_ in iv:
        if cs is None or s_ > ce:
            if cs is not None:
                union += ce - cs
            cs, ce = s_, e_
        else:
            ce = max(ce, e_)
    if cs is not None:
        union += ce - cs
    print('any-queue busy %.1f us/step (%.1f%%), all-idle %.1f us/step'
          % (union / 1e3 / nsteps, 100 * union / 1e3 / nsteps / wall, wall - union / 1e3 / nsteps))
    def table(rows, top):
        names = defaultdict(lambda: [0, 0])
        for r in rows:
            n = r['Kernel_Name'].replace('(anonymous namespace)::', '').replace('void ', '')
            n = n.split('(')[0][:60]
            names[n][0] += 1
            names[n][1] += r['e'] - r['s']
        print('%-62s %8s %10s' % ('kernel', 'n/step', 'us/step'))
        for n, (c, d) in sorted(names.items(), key=lambda x: -x[1][1])[:top]:
            print('%-62s %8.1f %10.1f' % (n, c / nsteps, d / 1e3 / nsteps))
    table(win, 30)
    for q, ks in sorted(byq.items()):
        print('--- queue %s' % q)
        table(ks, 15)


if __name__ == '__main__':
    main()
