"""Native MI355X engine (HIP kernels + HIP graphs). Filled in by engine/native.py."""


def native_supported(net):
    try:
        from .native import supports
    except ImportError:
        return False
    return supports(net)


def NativeTrainer(*a, **k):
    from .native import NativeTrainer as _NT
    return _NT(*a, **k)
