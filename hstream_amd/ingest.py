"""ctypes binding of the host ingest of libhstream_gpu (include/hstream_ingest.h).

``KeyDict`` is the native group-key dictionary (Aeson Value equality, ids in
first-seen order); ``Decoder`` turns a poll batch of JSON record values into
the columnar arrays of an ``hsg_batch`` in one call, over host threads. Both
run without a GPU. There is no Python fallback: the library must be built.
"""
import ctypes as C
import json
from typing import Sequence, Tuple

import numpy as np

from . import abi
from .engine import load_library

_declared = False


def _lib():
    global _declared
    L = load_library()
    if not _declared:
        vp, P = C.c_void_p, C.POINTER
        L.hsg_keydict_create.argtypes = [P(vp)]
        L.hsg_keydict_create.restype = C.c_int
        L.hsg_keydict_destroy.argtypes = [vp]
        L.hsg_keydict_destroy.restype = None
        L.hsg_keydict_size.argtypes = [vp]
        L.hsg_keydict_size.restype = C.c_uint64
        L.hsg_keydict_encode.argtypes = [vp, C.c_char_p, C.c_size_t, P(C.c_uint32)]
        L.hsg_keydict_encode.restype = C.c_int
        L.hsg_keydict_text.argtypes = [vp, C.c_uint32, C.c_char_p, C.c_size_t, P(C.c_size_t)]
        L.hsg_keydict_text.restype = C.c_int
        L.hsg_decoder_create.argtypes = [P(abi.hsg_decoder_config), P(vp)]
        L.hsg_decoder_create.restype = C.c_int
        L.hsg_decoder_destroy.argtypes = [vp]
        L.hsg_decoder_destroy.restype = None
        L.hsg_decode_json.argtypes = [vp, vp, C.c_uint64, C.c_char_p, vp, vp, vp, vp, P(vp), P(vp), vp,
                                      P(C.c_uint64), C.c_int]
        L.hsg_decode_json.restype = C.c_int
        L.hsg_decode_json_spelled.argtypes = [vp, vp, C.c_uint64, C.c_char_p, vp, vp, vp, vp, P(vp), P(vp), vp,
                                              P(C.c_uint64), vp, C.c_int]
        L.hsg_decode_json_spelled.restype = C.c_int
        L.hsg_keydict_spelling_text.argtypes = [vp, C.c_uint32, C.c_char_p, C.c_size_t, P(C.c_size_t)]
        L.hsg_keydict_spelling_text.restype = C.c_int
        _declared = True
    return L


def _check(rc, what):
    if rc != abi.HSG_OK:
        raise abi.HStreamGpuError(rc, what)


class KeyDict:
    """Group key <-> u32 id (hsg_keydict). ``encode`` takes a JSON text (or a
    Python value, serialised first); ``text`` / ``decode`` give back the key's
    Aeson encoding / its value."""

    def __init__(self):
        self._L = _lib()
        h = C.c_void_p()
        _check(self._L.hsg_keydict_create(C.byref(h)), "hsg_keydict_create")
        self._h = h

    def __len__(self):
        return int(self._L.hsg_keydict_size(self._h))

    def encode_json(self, text) -> int:
        b = text.encode() if isinstance(text, str) else bytes(text)
        out = C.c_uint32()
        _check(self._L.hsg_keydict_encode(self._h, b, len(b), C.byref(out)), "hsg_keydict_encode")
        return int(out.value)

    def encode(self, value) -> int:
        return self.encode_json(json.dumps(value))

    def text(self, i: int) -> str:
        n = C.c_size_t()
        rc = self._L.hsg_keydict_text(self._h, int(i), None, 0, C.byref(n))
        if rc not in (abi.HSG_OK, abi.HSG_E_CAPACITY):
            _check(rc, "hsg_keydict_text")
        buf = C.create_string_buffer(max(1, n.value))
        _check(self._L.hsg_keydict_text(self._h, int(i), buf, n.value, C.byref(n)), "hsg_keydict_text")
        return buf.raw[: n.value].decode()

    def decode(self, i: int):
        return json.loads(self.text(i))

    def spelling_text(self, spell: int) -> str:
        """Text of a record's key spelling (Decoder.decode(..., spellings=True))."""
        n = C.c_size_t()
        rc = self._L.hsg_keydict_spelling_text(self._h, int(spell), None, 0, C.byref(n))
        if rc not in (abi.HSG_OK, abi.HSG_E_CAPACITY):
            _check(rc, "hsg_keydict_spelling_text")
        buf = C.create_string_buffer(max(1, n.value))
        _check(self._L.hsg_keydict_spelling_text(self._h, int(spell), buf, n.value, C.byref(n)),
               "hsg_keydict_spelling_text")
        return buf.raw[: n.value].decode()

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            self._L.hsg_keydict_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Decoder:
    """hsg_decoder: GROUP BY field + aggregated fields -> columns.

    cols: [(field, hsg_col_type, numeric)] in the op's column order; numeric
    = the column feeds SUM/MIN/MAX/AVG/LAST (a value must be a Number), else
    COUNT(col) only (any present value counts). literal_forms: valid bytes
    carry bit 1 for numbers written with a negative exponent (ops with
    HSG_OPF_LITERAL_FORMS)."""

    def __init__(self, key_field: str, cols: Sequence[Tuple[str, int, bool]], literal_forms: bool = False):
        self._L = _lib()
        self.key_field = key_field
        self.cols = list(cols)
        n = len(self.cols)
        self._fields = (C.c_char_p * max(1, n))(*[f.encode() for f, _, _ in self.cols])
        self._types = (C.c_int32 * max(1, n))(*[t for _, t, _ in self.cols])
        self._num = (C.c_uint8 * max(1, n))(*[1 if num else 0 for _, _, num in self.cols])
        cfg = abi.hsg_decoder_config(key_field=key_field.encode(), n_cols=n, col_fields=self._fields,
                                     col_types=self._types, col_numeric=self._num,
                                     literal_forms=1 if literal_forms else 0)
        h = C.c_void_p()
        _check(self._L.hsg_decoder_create(C.byref(cfg), C.byref(h)), "hsg_decoder_create")
        self._h = h

    def decode(self, keys: KeyDict, buf: bytes, off: np.ndarray, ts: np.ndarray, threads: int = 0,
               spellings: bool = False):
        """One poll batch: buf holds the record values back to back, record i
        at buf[off[i]:off[i+1]]. Returns (key_id u32[n], ts i64[n], cols,
        valid, status u8[n], rejected), and with spellings=True also spell
        u32[n] (hsg_decode_json_spelled: each record's key spelling)."""
        n = len(off) - 1
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ts_in = np.ascontiguousarray(ts, dtype=np.int64)
        key = np.empty(n, np.uint32)
        ts_out = np.empty(n, np.int64)
        cols = [np.empty(n, np.float64 if t == abi.HSG_F64 else np.int64) for _, t, _ in self.cols]
        valid = [np.empty(n, np.uint8) for _ in self.cols]
        status = np.empty(n, np.uint8)
        cp = (C.c_void_p * max(1, len(cols)))(*[c.ctypes.data for c in cols])
        vp = (C.c_void_p * max(1, len(valid)))(*[v.ctypes.data for v in valid])
        rej = C.c_uint64()
        if spellings:
            spell = np.empty(n, np.uint32)
            _check(self._L.hsg_decode_json_spelled(self._h, keys.handle, n, buf, off.ctypes.data, ts_in.ctypes.data,
                                                   key.ctypes.data, ts_out.ctypes.data, cp, vp, status.ctypes.data,
                                                   C.byref(rej), spell.ctypes.data, int(threads)),
                   "hsg_decode_json_spelled")
            return key, ts_out, cols, valid, status, int(rej.value), spell
        _check(self._L.hsg_decode_json(self._h, keys.handle, n, buf, off.ctypes.data, ts_in.ctypes.data,
                                       key.ctypes.data, ts_out.ctypes.data, cp, vp, status.ctypes.data,
                                       C.byref(rej), int(threads)), "hsg_decode_json")
        return key, ts_out, cols, valid, status, int(rej.value)

    def close(self):
        if self._h:
            self._L.hsg_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def pack_records(values: Sequence[bytes]):
    """Record values -> (buffer, offsets) as hsg_decode_json takes them."""
    lens = np.fromiter((len(v) for v in values), dtype=np.uint64, count=len(values))
    off = np.zeros(len(values) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    return b"".join(values), off
