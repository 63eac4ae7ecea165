"""In-tree build of the HIP extension ``mercury_amd/_C*.so`` for gfx950.

Every ``csrc/*.hip`` is compiled with ``hipcc --offload-arch=gfx950`` (no
PyTorch headers, no hipify, no CUDA paths) and linked with the pybind11 binding
layer into one shared object next to this file, so it travels with the repo to
the GPU box and is what ``import mercury_amd.ops`` loads.  Objects are cached
in ``build/obj`` and rebuilt when a source or any header is newer.

    python -m mercury_amd._build            # build (parallel)
    python -m mercury_amd._build --clean
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'csrc')
OBJ = os.path.join(ROOT, 'build', 'obj')
ARCH = os.environ.get('PYTORCH_ROCM_ARCH', 'gfx950').split(';')[0]
ROCM = os.environ.get('ROCM_PATH', '/opt/rocm')
HIPCC = os.environ.get('HIPCC', os.path.join(ROCM, 'bin', 'hipcc'))
EXT_SUFFIX = sysconfig.get_config_var('EXT_SUFFIX') or '.so'
TARGET = os.path.join(ROOT, 'mercury_amd', '_C' + EXT_SUFFIX)

HIP_FLAGS = ['-O3', '-std=c++17', '-fPIC', '--offload-arch=' + ARCH, '-munsafe-fp-atomics',
             '-Wno-unused-result', '-I' + CSRC]


def _pybind_includes():
    import pybind11
    return ['-I' + pybind11.get_include(), '-I' + sysconfig.get_paths()['include']]


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, '*.h'))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _needs(src, obj, hdr_t):
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return os.path.getmtime(src) > t or hdr_t > t


def _compile(src, obj, extra):
    cmd = [HIPCC] + HIP_FLAGS + extra + ['-c', src, '-o', obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError('compile failed: %s\n%s\n%s' % (' '.join(cmd), r.stdout, r.stderr))
    return obj


def build(verbose=True, jobs=None):
    os.makedirs(OBJ, exist_ok=True)
    hdr_t = _newest_header()
    jobs = jobs or min(8, os.cpu_count() or 4)
    srcs = sorted(glob.glob(os.path.join(CSRC, '*.hip')))
    work = []
    objs = []
    for s in srcs:
        o = os.path.join(OBJ, os.path.basename(s) + '.o')
        objs.append(o)
        if _needs(s, o, hdr_t):
            work.append((s, o, []))
    b = os.path.join(CSRC, 'bindings.cpp')
    bo = os.path.join(OBJ, 'bindings.cpp.o')
    objs.append(bo)
    if _needs(b, bo, hdr_t):
        work.append((b, bo, _pybind_includes()))
    if work:
        if verbose:
            print('[mercury_amd] compiling %d file(s) for %s' % (len(work), ARCH), flush=True)
        with ThreadPoolExecutor(jobs) as ex:
            list(ex.map(lambda w: _compile(*w), work))
    if work or not os.path.exists(TARGET) or any(
            os.path.getmtime(o) > os.path.getmtime(TARGET) for o in objs):
        # librccl.so.1 resolves at import to the RCCL torch already loaded (same soname)
        cmd = ([HIPCC, '-shared', '-fPIC', '--offload-arch=' + ARCH] + objs +
               ['-L' + os.path.join(ROCM, 'lib'), '-lrccl', '-o', TARGET])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('link failed: %s\n%s' % (r.stdout, r.stderr))
        if verbose:
            print('[mercury_amd] built %s' % os.path.relpath(TARGET, ROOT), flush=True)
    return TARGET


TOOLS = os.path.join(ROOT, 'mercury_amd', '_tools.so')


def build_tools(verbose=True):
    """Diagnostic kernels (``csrc/tools/*.hip``, C ABI, loaded by ctypes from ``bench/``) in a
    shared object of their own, so nothing of them ships in the production extension."""
    srcs = sorted(glob.glob(os.path.join(CSRC, 'tools', '*.hip')))
    if not srcs:
        return None
    hdr_t = _newest_header()
    objs = []
    for s in srcs:
        o = os.path.join(OBJ, 'tools_' + os.path.basename(s) + '.o')
        objs.append(o)
        if _needs(s, o, hdr_t):
            _compile(s, o, [])
    if not os.path.exists(TOOLS) or any(os.path.getmtime(o) > os.path.getmtime(TOOLS)
                                        for o in objs):
        cmd = [HIPCC, '-shared', '-fPIC', '--offload-arch=' + ARCH] + objs + ['-o', TOOLS]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError('link failed: %s\n%s' % (r.stdout, r.stderr))
        if verbose:
            print('[mercury_amd] built %s' % os.path.relpath(TOOLS, ROOT), flush=True)
    return TOOLS


def clean():
    for f in glob.glob(os.path.join(OBJ, '*.o')) + [TARGET, TOOLS]:
        if os.path.exists(f):
            os.remove(f)


if __name__ == '__main__':
    if '--clean' in sys.argv:
        clean()
    build()
    build_tools()
