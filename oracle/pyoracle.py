"""ORACLE binding — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/libhsoracle.so (the C++ restatement in hsoracle.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product package never does.
"""
import ctypes as C
import os
import subprocess

from hstream_amd import abi
from hstream_amd.columnar import OpHandle, OpSpec, declare_op_functions

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libhsoracle.so")
_lib = None


def build(force=False):
    if force or not os.path.exists(_LIB_PATH) or (
        os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "hsoracle.cpp"))
    ):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        declare_op_functions(L, "hso")
        L.hso_op_create_ex.argtypes = [C.POINTER(abi.hsg_op_config), C.c_int, C.POINTER(C.c_void_p)]
        L.hso_op_create_ex.restype = C.c_int
        L.hso_windows_for.argtypes = [C.c_int64, C.c_int64, C.c_int64, C.POINTER(C.c_int64), C.c_int]
        L.hso_windows_for.restype = C.c_int
        _lib = L
    return _lib


class OracleOp(OpHandle):
    def __init__(self, spec: OpSpec, faithful_sessions=True):
        L = lib()
        cfg, keep = spec.to_config()
        h = C.c_void_p()
        rc = L.hso_op_create_ex(C.byref(cfg), 1 if faithful_sessions else 0, C.byref(h))
        if rc != abi.HSG_OK:
            raise abi.HStreamGpuError(rc, "hso_op_create")
        super().__init__(L, "hso", h, spec)


def windows_for(ts, size, adv):
    L = lib()
    buf = (C.c_int64 * 4096)()
    n = L.hso_windows_for(ts, size, adv, buf, 4096)
    return [(buf[i], buf[i] + size) for i in range(min(n, 4096))]
