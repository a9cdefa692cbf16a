"""ctypes binding of the GPU stream-stream join (include/hstream_join.h)."""
import ctypes as C

import numpy as np

from . import abi
from .engine import load_library

_declared = False


def _lib():
    global _declared
    L = load_library()
    if not _declared:
        vp, P = C.c_void_p, C.POINTER
        L.hsg_join_create.argtypes = [vp, P(abi.hsg_join_config), P(vp)]
        L.hsg_join_create.restype = C.c_int
        L.hsg_join_destroy.argtypes = [vp]
        L.hsg_join_destroy.restype = None
        L.hsg_join_last_error.argtypes = [vp]
        L.hsg_join_last_error.restype = C.c_char_p
        L.hsg_join_push.argtypes = [vp, P(abi.hsg_join_batch)]
        L.hsg_join_push.restype = C.c_int
        L.hsg_join_pending.argtypes = [vp, P(C.c_uint64)]
        L.hsg_join_pending.restype = C.c_int
        L.hsg_join_drain.argtypes = [vp, P(abi.hsg_join_rows), P(C.c_uint64)]
        L.hsg_join_drain.restype = C.c_int
        L.hsg_join_state_rows.argtypes = [vp, P(C.c_uint64)]
        L.hsg_join_state_rows.restype = C.c_int
        _declared = True
    return L


class Join:
    """joinStream over one engine: push poll batches of both streams, drain
    (this handle, other handle, join key, ts) rows."""

    def __init__(self, engine, before_ms, after_ms, batch_capacity=1 << 20):
        self._L = _lib()
        cfg = abi.hsg_join_config(before_ms=before_ms, after_ms=after_ms, batch_capacity=batch_capacity)
        h = C.c_void_p()
        self._check(self._L.hsg_join_create(engine._h, C.byref(cfg), C.byref(h)), "hsg_join_create", None)
        self._h = h

    def _check(self, rc, what, h="self"):
        if rc != abi.HSG_OK:
            msg = ""
            if h is not None and getattr(self, "_h", None):
                msg = (self._L.hsg_join_last_error(self._h) or b"").decode()
            raise abi.HStreamGpuError(rc, f"{what}: {msg}")

    def push(self, side, key, join_key, ts, handle):
        side = np.ascontiguousarray(side, np.uint8)
        key = np.ascontiguousarray(key, np.uint32)
        jk = np.ascontiguousarray(join_key, np.uint32)
        ts = np.ascontiguousarray(ts, np.int64)
        hd = np.ascontiguousarray(handle, np.uint64)
        b = abi.hsg_join_batch(n=len(ts), mem=abi.HSG_MEM_HOST, side=side.ctypes.data, key_id=key.ctypes.data,
                               join_key=jk.ctypes.data, ts=ts.ctypes.data, handle=hd.ctypes.data)
        self._check(self._L.hsg_join_push(self._h, C.byref(b)), "hsg_join_push")

    def drain(self):
        n = C.c_uint64()
        self._check(self._L.hsg_join_pending(self._h, C.byref(n)), "hsg_join_pending")
        m = n.value
        th, oh, jk, ts = (np.empty(m, np.uint64), np.empty(m, np.uint64), np.empty(m, np.uint32),
                          np.empty(m, np.int64))
        r = abi.hsg_join_rows(capacity=m, mem=abi.HSG_MEM_HOST, this_handle=th.ctypes.data,
                              other_handle=oh.ctypes.data, join_key=jk.ctypes.data, ts=ts.ctypes.data)
        self._check(self._L.hsg_join_drain(self._h, C.byref(r), C.byref(n)), "hsg_join_drain")
        return th, oh, jk, ts

    def state_rows(self):
        n = C.c_uint64()
        self._check(self._L.hsg_join_state_rows(self._h, C.byref(n)), "hsg_join_state_rows")
        return n.value

    def close(self):
        if self._h:
            self._L.hsg_join_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
