"""Per-dispatch sequence of one step from a rocprofv3 ``--kernel-trace`` capture.

    python bench/seq_trace.py <rocprof out dir> [marker_kernel] [n_steps]

Takes the last ``n_steps`` windows that each start at a launch of the marker kernel
(default ``step_begin_kernel``: once per train-graph replay) and prints, in launch
order, every dispatch of the window with its grid, workgroup size, duration and the
gap since the previous dispatch ended -- the median over the windows -- so each conv /
BN pass of the step can be named and priced (which layer is slow, where launch gaps
sit).  Used on ``bench.py --replay-only train`` traces, where one queue holds the step.
"""
import csv
import glob
import statistics
import sys


def main():
    root = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'step_begin_kernel'
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    f = glob.glob(root + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        r['s'] = int(r['Start_Timestamp'])
        r['e'] = int(r['End_Timestamp'])
    rows.sort(key=lambda r: r['s'])
    starts = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    if len(starts) < 2:
        print('fewer than two marker launches')
        return
    starts = starts[-(nsteps + 1):]
    wins = [rows[a:b] for a, b in zip(starts[:-1], starts[1:])]
    n = min(len(w) for w in wins)
    wins = [w for w in wins if len(w) == n]
    gk = 'Grid_Size' if 'Grid_Size' in rows[0] else 'Grid_Size_X'
    wk = 'Workgroup_Size' if 'Workgroup_Size' in rows[0] else 'Workgroup_Size_X'
    tot = 0.0
    print('%d windows of %d dispatches' % (len(wins), n))
    print('%3s %9s %8s %6s %7s  %s' % ('#', 'grid', 'wg', 'us', 'gap', 'kernel'))
    for j in range(n):
        d = statistics.median((w[j]['e'] - w[j]['s']) / 1e3 for w in wins)
        g = statistics.median(((w[j]['s'] - w[j - 1]['e']) / 1e3) if j else 0.0 for w in wins)
        tot += d
        r = wins[-1][j]
        name = r['Kernel_Name']
        name = name[:70]
        print('%3d %9s %8s %6.1f %7.1f  %s' % (j, r.get(gk, ''), r.get(wk, ''), d, g, name))
    wall = statistics.median((w[-1]['e'] - w[0]['s']) / 1e3 for w in wins)
    print('sum of dispatch medians %.1f us, window wall %.1f us' % (tot, wall))


if __name__ == '__main__':
    main()
