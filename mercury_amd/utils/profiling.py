"""roctx ranges / markers for rocprofv3 and a step-window profiler switch.

The reference times phases with ``time.time()`` and no device sync
(`pytorch_collab.py:129-168`), so its numbers are async-skewed and its "IS
time" is empty.  Here:

* ``range(name)`` / ``mark(name)`` emit roctx ranges straight from the
  rocprofiler-sdk roctx library (ctypes; no-ops when it is absent), so
  ``rocprofv3 --marker-trace`` attributes kernels to ``score`` / ``train`` /
  ``allreduce`` / ``tail`` phases of each step;
* ``StepWindow`` opens a ``mercury_profile`` range around steps
  ``[start, start+n)`` of a run (``Config.profile_steps``/``profile_start``),
  which is the window a marker-filtered rocprofv3 run keeps;
* device-accurate phase times come from ``utils.logging.PhaseTimer`` (HIP
  events), not from host clocks.
"""
from __future__ import annotations

import contextlib
import ctypes
import ctypes.util
import os

_LIB = None
_TRIED = False


def _lib():
    global _LIB, _TRIED
    if _TRIED:
        return _LIB
    _TRIED = True
    root = os.path.join(os.environ.get('ROCM_PATH', '/opt/rocm'), 'lib')
    # the rocprofiler-sdk roctx is what rocprofv3 --marker-trace intercepts; legacy roctx64 next
    cands = [os.path.join(root, 'librocprofiler-sdk-roctx.so'), os.path.join(root, 'libroctx64.so'),
             ctypes.util.find_library('roctx64') or '']
    for c in cands:
        if c and os.path.exists(c):
            try:
                lib = ctypes.CDLL(c)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _LIB = lib
                break
            except OSError:
                continue
    return _LIB


def available():
    return _lib() is not None


def push(name):
    lib = _lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())


def pop():
    lib = _lib()
    if lib is not None:
        lib.roctxRangePop()


def mark(name):
    lib = _lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())


@contextlib.contextmanager
def range(name, enabled=True):   # noqa: A001 - mirrors the roctx API name
    if not enabled:
        yield
        return
    push(name)
    try:
        yield
    finally:
        pop()


class StepWindow(object):
    """Open a ``mercury_profile`` roctx range over steps ``[start, start + n)``."""

    def __init__(self, start=0, n=0):
        self.start, self.n = int(start), int(n)
        self.open = False

    def step(self, i):
        if self.n <= 0:
            return
        if not self.open and i == self.start:
            push('mercury_profile')
            self.open = True
        elif self.open and i == self.start + self.n:
            pop()
            self.open = False

    def close(self):
        if self.open:
            pop()
            self.open = False
