"""Instruction mix of a kernel's hottest loops from hipcc's device assembly.

    python bench/asm_loop.py csrc/igemm.hip '_ZN12_GLOBAL__N_115igemm_nt_kernelILi256ELi64ELb0E'

Compiles the file for gfx950 to assembly and prints, for the two loops with the most basic
blocks, the count of MFMA / VALU / SALU / LDS / VMEM instructions and of vmcnt(0) waits.
"""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    out = os.path.join(tempfile.mkdtemp(), 'k.s')
    subprocess.run(['/opt/rocm/bin/hipcc', '-O3', '-std=c++17', '--offload-arch=gfx950',
                    '-munsafe-fp-atomics', '-I' + os.path.join(ROOT, 'csrc'), '-S',
                    '--cuda-device-only', src, '-o', out], check=True, capture_output=True)
    s = open(out).read()
    names = sorted(set(n for n in re.findall(r'^(\S+):', s, re.M) if n.startswith(prefix)))
    for name in names[:2]:
        i = s.index(name + ':')
        j = s.index('.Lfunc_end', i)
        txt = s[i:j]
        body = txt.splitlines()
        hdrs = collections.Counter(re.findall(r'Loop: Header=(BB\d+_\d+) Depth=1', txt))
        print(name)
        for h, _ in hdrs.most_common(2):
            blk, inloop = [], False
            for line in body:
                m = re.match(r'^(\.LBB\d+_\d+):\s*(;.*)?$', line)
                if m:
                    inloop = ('Header=%s' % h in line) or m.group(1) == '.L' + h
                if inloop:
                    blk.append(line)
            cnt = collections.Counter()
            for line in blk:
                t = line.strip().split()
                if not t or t[0].startswith((';', '.')):
                    continue
                op = t[0]
                cls = ('mfma' if 'mfma' in op else 'valu' if op.startswith('v_') else
                       'salu' if op.startswith('s_') else 'lds' if op.startswith('ds_') else
                       'vmem' if op.startswith(('global_', 'buffer_')) else op)
                cnt[cls] += 1
            print('  loop %s: %s  vmcnt(0) waits: %d' % (h, dict(cnt),
                                                        sum('vmcnt(0)' in x for x in blk)))


if __name__ == '__main__':
    main()
