"""Optional roctx phase ranges around the WAM call's stages (SURVEY §5 profiling; the reference has
none). Off unless WAM_PROFILE=1 is set in the environment: then every stage of a call
(noise + analysis, synthesis, model, adjoint + maps, accumulate, collectives) is bracketed by a
roctxRangePush/Pop that `rocprofv3 --marker-trace` records beside the kernel trace, e.g.

    WAM_PROFILE=1 rocprofv3 --marker-trace --kernel-trace --stats -d out -- python bench.py ...

Ranges are host-side markers: they cost two C calls per stage and nothing on the GPU.
"""
import contextlib
import ctypes
import os

_LIB = None
ENABLED = os.environ.get("WAM_PROFILE", "0") not in ("", "0")


def _lib():
    global _LIB
    if _LIB is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "/opt/rocm/lib/librocprofiler-sdk-roctx.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _LIB = lib
                break
            except (OSError, AttributeError):
                continue
        else:
            _LIB = False
    return _LIB


@contextlib.contextmanager
def _range(name):
    lib = _lib()
    if lib:
        lib.roctxRangePushA(("wam:" + name).encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def phase(name):
    """Context manager: a roctx range named wam:<name> when WAM_PROFILE=1, else a no-op."""
    return _range(name) if ENABLED else contextlib.nullcontext()
