"""Per-kernel summary of a rocprofv3 SQLite (rocpd) output: calls, total ms, average us and
share of kernel time, sorted by total time.

    python bench/rocpd_sum.py <dir with *_results.db> [top N] [--csv out.csv]
"""
import csv
import glob
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    out_csv = sys.argv[sys.argv.index('--csv') + 1] if '--csv' in sys.argv else None
    if out_csv in args:
        args.remove(out_csv)
    db = glob.glob(args[0] + '/**/*.db', recursive=True)[0]
    top = int(args[1]) if len(args) > 1 else 30
    c = sqlite3.connect(db)
    rows = c.execute('select name, count(*), sum(duration), avg(duration) from kernels '
                     'group by name order by sum(duration) desc').fetchall()
    tot = sum(r[2] for r in rows) or 1
    if out_csv:
        with open(out_csv, 'w', newline='') as f:
            w = csv.writer(f)
            w.writerow(['kernel', 'calls', 'total_ms', 'avg_us', 'pct'])
            for n, k, s, a in rows:
                w.writerow([n, k, s / 1e6, a / 1e3, 100.0 * s / tot])
    print('%-70s %7s %9s %8s %5s' % ('kernel', 'calls', 'total_ms', 'avg_us', 'pct'))
    for n, k, s, a in rows[:top]:
        print('%-70s %7d %9.2f %8.2f %5.1f' % (n[:70], k, s / 1e6, a / 1e3, 100.0 * s / tot))
    print('kernels %d, total kernel time %.2f ms' % (sum(r[1] for r in rows), tot / 1e6))


if __name__ == '__main__':
    main()
