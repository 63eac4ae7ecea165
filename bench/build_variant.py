"""Build the extension from another git revision of chosen csrc files, for in-process A/B runs.

    python bench/build_variant.py REV OUT.so csrc/igemm.hip csrc/igemm.h csrc/bindings.cpp
    MERCURY_EXT_PATH=OUT.so python bench.py ...
    MERCURY_VARIANT_FLAGS=-DMERCURY_STAMPS python bench/build_variant.py HEAD OUT.so   # + flags

Files not named come from the working tree.  Kernel timings differ by several percent
between MI355X devices, so variants are compared on the same box in one GPU call.
"""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    rev, out, files = sys.argv[1], os.path.abspath(sys.argv[2]), sys.argv[3:]
    from mercury_amd import _build
    tmp = tempfile.mkdtemp()
    src = os.path.join(tmp, 'csrc')
    shutil.copytree(os.path.join(ROOT, 'csrc'), src)
    for f in files:
        data = subprocess.run(['git', 'show', '%s:%s' % (rev, f)], cwd=ROOT, check=True,
                              capture_output=True).stdout
        with open(os.path.join(tmp, f), 'wb') as fh:
            fh.write(data)
    _build.CSRC, _build.OBJ, _build.TARGET = src, os.path.join(tmp, 'obj'), out
    _build.HIP_FLAGS = [f if not f.startswith('-I') else '-I' + src for f in _build.HIP_FLAGS]
    _build.HIP_FLAGS += os.environ.get('MERCURY_VARIANT_FLAGS', '').split()
    _build.build(verbose=True)
    print(out)


if __name__ == '__main__':
    main()
