"""ORACLE binding — TEST INFRASTRUCTURE ONLY.

ctypes binding of oracle/libhsoracle.so (the C++ restatement in hsoracle.cpp).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module; the product package never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

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
        L.hso_push_batch_ex.argtypes = [C.c_void_p, C.POINTER(abi.hsg_batch), C.POINTER(C.c_int64), C.c_void_p,
                                        C.c_void_p]
        L.hso_push_batch_ex.restype = C.c_int
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

    def push_ex(self, key_id, ts, cols=(), valid=None, watermark=-1, rec_wm=None, seq=None):
        """push with explicit per-record stream time / global sequence numbers."""
        from hstream_amd.columnar import make_batch
        b, keep = make_batch(key_id, ts, cols, valid)
        rw = None if rec_wm is None else np.ascontiguousarray(rec_wm, dtype=np.int64)
        sq = None if seq is None else np.ascontiguousarray(seq, dtype=np.int64)
        wm = C.c_int64(watermark)
        rc = self._lib.hso_push_batch_ex(self._h, C.byref(b), C.byref(wm),
                                         None if rw is None else rw.ctypes.data,
                                         None if sq is None else sq.ctypes.data)
        del keep
        self._check(rc, "push_batch_ex")
        return wm.value


def windows_for(ts, size, adv):
    L = lib()
    buf = (C.c_int64 * 4096)()
    n = L.hso_windows_for(ts, size, adv, buf, 4096)
    return [(buf[i], buf[i] + size) for i in range(min(n, 4096))]
