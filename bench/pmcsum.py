"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel name.

    python bench/pmcsum.py gpurun_out/pmc_step/p1 [top]

Prints, per kernel (summed over dispatches), each counter plus MFMA-busy / busy-cycle and
LDS-conflict / LDS-instruction ratios when those counters are present.  SQ_VALU_MFMA_BUSY_CYCLES
is summed over more units than SQ_BUSY_CYCLES, so that ratio exceeds 1: compare it between
kernels, not against 1.
"""
import csv
import glob
import sys
from collections import defaultdict


def main():
    f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:70]
        acc[k][r['Counter_Name']] += float(r['Counter_Value'])
        disp[k].add(r['Dispatch_Id'])
    names = sorted({c for v in acc.values() for c in v})
    rows = sorted(acc.items(), key=lambda kv: -kv[1].get('SQ_BUSY_CYCLES', 0))[:top]
    for k, v in rows:
        extra = []
        if v.get('SQ_BUSY_CYCLES'):
            extra.append('mfma_busy/busy(raw)=%.3f' % (v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / v['SQ_BUSY_CYCLES']))
        if v.get('SQ_INSTS_MFMA'):
            extra.append('valu/mfma=%.2f' % (v.get('SQ_INSTS_VALU', 0) / v['SQ_INSTS_MFMA']))
        if v.get('SQ_INSTS_LDS'):
            extra.append('lds_conflict/lds_inst=%.3f' % (v.get('SQ_LDS_BANK_CONFLICT', 0) / v['SQ_INSTS_LDS']))
        print('%-70s n=%-5d %s' % (k, len(disp[k]), ' '.join(extra)))
        print('    ' + ' '.join('%s=%.3g' % (c, v[c]) for c in names if c in v))


if __name__ == '__main__':
    main()
