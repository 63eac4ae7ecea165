"""Which kernels stretch when the scoring and training streams overlap.

    python bench/overlap_stretch.py <overlapped trace dir> <train-solo dir> <score-solo dir>

Each argument is a rocprofv3 ``--kernel-trace --output-format csv`` directory of ``bench.py``:
the normal timed run (both streams), and ``--replay-only train`` / ``--replay-only score``.
Kernels are matched by (queue role, position in the per-step sequence); the report lists, per
stream, every position's solo and overlapped median duration and the stretch, sorted by the
absolute time added -- where the overlapped step loses its time.
"""
import csv
import glob
import statistics as st
import sys
from collections import defaultdict


def load(root):
    f = glob.glob(root + '/**/*kernel_trace.csv', recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    for r in rows:
        r['s'] = int(r['Start_Timestamp'])
        r['e'] = int(r['End_Timestamp'])
        r['q'] = r.get('Queue_Id') or r.get('Stream_Id')
    rows.sort(key=lambda r: r['s'])
    return rows


def periods(rows, first, n_min=5):
    """Split one queue's kernels into repetitions starting at a kernel named ``first``."""
    out, cur = [], None
    for r in rows:
        if first in r['Kernel_Name']:
            if cur:
                out.append(cur)
            cur = []
        if cur is not None:
            cur.append(r)
    return [p for p in out if len(p) >= n_min]


def seqs(rows, first):
    byq = defaultdict(list)
    for r in rows:
        byq[r['q']].append(r)
    best = None
    for q, ks in byq.items():
        ps = periods(ks, first)
        if ps and (best is None or len(ps) > len(best)):
            best = ps
    if not best:
        return None
    L = st.mode([len(p) for p in best])
    best = [p for p in best if len(p) == L][-30:]
    names = [k['Kernel_Name'][:70] for k in best[0]]
    dur = [st.median([(p[i]['e'] - p[i]['s']) / 1e3 for p in best]) for i in range(L)]
    return names, dur


def main():
    ov, tr, sc = (load(a) for a in sys.argv[1:4])
    for role, first, solo in (('train', 'step_begin', tr), ('score', 'pool_build', sc)):
        a, b = seqs(ov, first), seqs(solo, first)
        if not a or not b:
            print(role, ': sequence not found')
            continue
        (na, da), (nb, db) = a, b
        if len(na) != len(nb):
            print(role, ': sequence lengths differ', len(na), len(nb))
        n = min(len(na), len(nb))
        rows = [(da[i] - db[i], i, na[i], db[i], da[i]) for i in range(n)]
        print('%s: %d kernels, solo %.1f us, overlapped %.1f us (sum of medians)'
              % (role, n, sum(db[:n]), sum(da[:n])))
        for add, i, name, s0, s1 in sorted(rows, reverse=True)[:25]:
            print('  #%-3d +%6.1f us  solo %6.1f  overlapped %6.1f  x%.2f  %s'
                  % (i, add, s0, s1, s1 / max(s0, 1e-3), name))


if __name__ == '__main__':
    main()
