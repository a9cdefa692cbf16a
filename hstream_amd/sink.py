"""ctypes binding of the GPU sink encoder (include/hstream_sink.h).

``Sink(op, keys, key_field, members, windowed)`` turns changelog rows into
the key / value bytes the reference's sink serdes produce; ``format_number``
is the host copy of the encoder's number formatter (for tests and hosts that
print single values the same way).
"""
import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np

from . import abi
from .abi import hsg_sink_config, hsg_sink_records
from .engine import load_library

_declared = False


def _lib():
    global _declared
    L = load_library()
    if not _declared:
        vp, P = C.c_void_p, C.POINTER
        L.hsg_sink_create.argtypes = [vp, vp, P(hsg_sink_config), P(vp)]
        L.hsg_sink_create.restype = C.c_int
        L.hsg_sink_destroy.argtypes = [vp]
        L.hsg_sink_destroy.restype = None
        L.hsg_sink_encode.argtypes = [vp, P(abi.hsg_rows), C.c_uint64, P(hsg_sink_records), P(C.c_uint64),
                                      P(C.c_uint64)]
        L.hsg_sink_encode.restype = C.c_int
        L.hsg_sink_encode_spelled.argtypes = [vp, P(abi.hsg_rows), C.c_uint64, P(abi.hsg_sink_spellings),
                                              P(hsg_sink_records), P(C.c_uint64), P(C.c_uint64)]
        L.hsg_sink_encode_spelled.restype = C.c_int
        L.hsg_sink_member_order.argtypes = [P(C.c_char_p), C.c_int32, P(C.c_int32)]
        L.hsg_sink_member_order.restype = C.c_int
        L.hsg_format_number.argtypes = [C.c_int32, C.c_int64, C.c_char_p, C.c_size_t, P(C.c_size_t)]
        L.hsg_format_number.restype = C.c_int
        _declared = True
    return L


def format_number(value, is_f64: bool, agg: str = "") -> str:
    """hsg_format_number; agg "sum" / "min" / "max": the double of that
    aggregate in a row without literal forms (its identity prints as the
    reference's initial value), else printed exactly."""
    L = _lib()
    bits = int(np.array([value], np.float64).view(np.int64)[0]) if is_f64 else int(value)
    buf = C.create_string_buffer(64)
    n = C.c_size_t()
    kind = {"": 1, "sum": 2, "min": 3, "max": 4}[agg] if is_f64 else 0
    rc = L.hsg_format_number(kind, bits, buf, 64, C.byref(n))
    if rc != abi.HSG_OK:
        raise abi.HStreamGpuError(rc, "hsg_format_number")
    return buf.raw[: n.value].decode()


def member_order(aliases: Sequence[str]) -> List[int]:
    """Indices of `aliases` in the order the encoder writes the value
    object's members (aeson's HashMap traversal order)."""
    L = _lib()
    n = len(aliases)
    arr = (C.c_char_p * max(1, n))(*[a.encode() for a in aliases])
    out = (C.c_int32 * max(1, n))()
    rc = L.hsg_sink_member_order(arr, n, out)
    if rc != abi.HSG_OK:
        raise abi.HStreamGpuError(rc, "hsg_sink_member_order")
    return list(out[:n])


class Sink:
    """members: [(alias, agg column or -1 for the GROUP BY value)], SELECT
    order; the encoder writes them in aeson's order (member_order)."""

    def __init__(self, op, keys, key_field: str, members: Sequence[Tuple[str, int]], windowed=True):
        self._L = _lib()
        self._keys = keys  # the dictionary must outlive the sink
        n = len(members)
        self._aliases = (C.c_char_p * max(1, n))(*[a.encode() for a, _ in members])
        self._idx = (C.c_int32 * max(1, n))(*[j for _, j in members])
        cfg = hsg_sink_config(windowed=1 if windowed else 0, n_members=n, key_field=key_field.encode(),
                              aliases=self._aliases, agg_index=self._idx)
        h = C.c_void_p()
        rc = self._L.hsg_sink_create(op._h, keys.handle, C.byref(cfg), C.byref(h))
        if rc != abi.HSG_OK:
            raise abi.HStreamGpuError(rc, "hsg_sink_create")
        self._h = h
        self.n_aggs = len(op.spec.aggs)

    def encode(self, rows, spellings=None, src_base: int = 0) -> List[Tuple[bytes, bytes]]:
        """Host rows (columnar.Rows) -> [(key bytes, value bytes)]. The rows'
        literal forms (rows.form) are used when present; spellings = the
        records' key spellings (Decoder.decode(..., spellings=True)) of the
        records whose global indices start at src_base
        (hsg_sink_encode_spelled)."""
        n = len(rows)
        key = np.ascontiguousarray(rows.key_id, np.uint32)
        ws = np.ascontiguousarray(rows.win_start, np.int64)
        src = np.ascontiguousarray(rows.src_index, np.int64)
        aggs = [np.ascontiguousarray(a).view(np.int64) for a in rows.aggs]
        ap = (C.c_void_p * max(1, len(aggs)))(*[a.ctypes.data for a in aggs])
        form = np.ascontiguousarray(rows.form, np.uint32) if rows.form is not None else None
        r = abi.hsg_rows(capacity=n, mem=abi.HSG_MEM_HOST, n_aggs=len(aggs), key_id=key.ctypes.data,
                         win_start=ws.ctypes.data, win_end=None, src_index=src.ctypes.data,
                         aggs=C.cast(ap, C.POINTER(C.c_void_p)),
                         form=form.ctypes.data if form is not None else None)
        sp = None
        if spellings is not None:
            spa = np.ascontiguousarray(spellings, np.uint32)
            sp = abi.hsg_sink_spellings(spell=spa.ctypes.data, n=len(spa), src_base=int(src_base),
                                        mem=abi.HSG_MEM_HOST)
            self._keep_sp = spa
        koff = np.zeros(n + 1, np.uint64)
        voff = np.zeros(n + 1, np.uint64)
        kneed, vneed = C.c_uint64(), C.c_uint64()
        out = hsg_sink_records(mem=abi.HSG_MEM_HOST, key_capacity=0, value_capacity=0, key_bytes=None,
                               key_off=koff.ctypes.data, value_bytes=None, value_off=voff.ctypes.data)
        rc = self._L.hsg_sink_encode_spelled(self._h, C.byref(r), n, C.byref(sp) if sp is not None else None,
                                             C.byref(out), C.byref(kneed), C.byref(vneed))
        if rc not in (abi.HSG_OK, abi.HSG_E_CAPACITY):
            raise abi.HStreamGpuError(rc, "hsg_sink_encode")
        kb = np.zeros(max(1, kneed.value), np.uint8)
        vb = np.zeros(max(1, vneed.value), np.uint8)
        out.key_capacity, out.value_capacity = kneed.value, vneed.value
        out.key_bytes, out.value_bytes = kb.ctypes.data, vb.ctypes.data
        rc = self._L.hsg_sink_encode_spelled(self._h, C.byref(r), n, C.byref(sp) if sp is not None else None,
                                             C.byref(out), C.byref(kneed), C.byref(vneed))
        if rc != abi.HSG_OK:
            raise abi.HStreamGpuError(rc, "hsg_sink_encode")
        kbb, vbb = kb.tobytes(), vb.tobytes()
        return [(kbb[koff[i]:koff[i + 1]], vbb[voff[i]:voff[i + 1]]) for i in range(n)]

    def close(self):
        if self._h:
            self._L.hsg_sink_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
