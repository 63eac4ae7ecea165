"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel name.

    python bench/pmcsum.py gpurun_out/pmc_step/p1 [top]

Prints, per kernel (summed over dispatches), the counters and the derived ratios the counters
of that pass allow:

* ``mfma_util``  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs * SIMDs): the fraction of
  every SIMD's cycles its matrix core was busy while the kernel ran (rocprofv3's ``MfmaUtil``
  expression; GRBM_GUI_ACTIVE is collected once per XCD, so its sum is divided by 8).  A kernel
  on half the CUs (the scoring convs' 128-block grids) tops out at 0.5;
* ``mfma_tflops`` = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 FLOP over the kernel's active time
  (GRBM_GUI_ACTIVE / 8 at 2.4 GHz, an upper clock bound: the figure is a lower bound);
* ``lds_conflict/lds_inst``, ``valu/mfma``, ``lds_wait/wave`` where their counters are present.
"""
import csv
import glob
import sys
from collections import defaultdict

XCDS, SIMDS, CLK = 8, 1024, 2.4e9


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
    key = 'GRBM_GUI_ACTIVE' if 'GRBM_GUI_ACTIVE' in names else 'SQ_BUSY_CYCLES'
    rows = sorted(acc.items(), key=lambda kv: -kv[1].get(key, 0))[:top]
    for k, v in rows:
        extra = []
        act = v.get('GRBM_GUI_ACTIVE', 0) / XCDS
        if act and 'SQ_VALU_MFMA_BUSY_CYCLES' in v:
            extra.append('mfma_util=%.3f' % (v['SQ_VALU_MFMA_BUSY_CYCLES'] / (act * SIMDS)))
        if act and 'SQ_INSTS_VALU_MFMA_MOPS_BF16' in v:
            extra.append('mfma_tflops>=%.0f' % (v['SQ_INSTS_VALU_MFMA_MOPS_BF16'] * 512 /
                                                (act / CLK) / 1e12))
        if act:
            extra.append('active_us=%.1f/disp' % (act / CLK * 1e6 / len(disp[k])))
        if v.get('SQ_INSTS_MFMA') and 'SQ_INSTS_VALU' in v:
            extra.append('valu/mfma=%.2f' % (v['SQ_INSTS_VALU'] / v['SQ_INSTS_MFMA']))
        if v.get('SQ_INSTS_LDS') and 'SQ_LDS_BANK_CONFLICT' in v:
            extra.append('lds_conflict/lds_inst=%.3f' % (v['SQ_LDS_BANK_CONFLICT'] / v['SQ_INSTS_LDS']))
        if v.get('SQ_WAVE_CYCLES') and 'SQ_WAIT_INST_LDS' in v:
            extra.append('lds_wait/wave=%.3f' % (v['SQ_WAIT_INST_LDS'] / v['SQ_WAVE_CYCLES']))
        if v.get('SQ_WAVE_CYCLES') and 'SQ_WAIT_ANY' in v:
            extra.append('wait_any/wave=%.3f' % (v['SQ_WAIT_ANY'] / v['SQ_WAVE_CYCLES']))
        print('%-70s n=%-5d %s' % (k, len(disp[k]), ' '.join(extra)))
        print('    ' + ' '.join('%s=%.3g' % (c, v[c]) for c in names if c in v))


if __name__ == '__main__':
    main()
