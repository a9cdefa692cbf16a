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
        L.hsg_decode_json_batch.argtypes = [vp, vp, C.c_uint64, C.c_char_p, vp, vp, P(abi.hsg_decode_buffers),
                                            P(abi.hsg_batch), vp, P(C.c_uint64), vp, C.c_int]
        L.hsg_decode_json_batch.restype = C.c_int
        L.hsg_batch_narrow.argtypes = [P(abi.hsg_batch), vp, C.c_uint32, vp, P(C.c_uint32), C.c_int]
        L.hsg_batch_narrow.restype = C.c_int
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

    def decode_batch(self, keys: KeyDict, buf: bytes, off: np.ndarray, ts: np.ndarray, allow: int = abi.HSG_NARROW_ALL,
                     threads: int = 0, spellings: bool = False, alloc=None):
        """One poll batch straight into a ready hsg_batch
        (hsg_decode_json_batch): decoded, then narrowed in place to the
        narrowest lossless transport `allow` permits (hsg_batch_narrow).
        alloc(nbytes) -> (numpy uint8 view, owner) lets the caller put the
        arrays in pinned memory for hsg_push_batch_async. Returns a
        DecodedBatch."""
        n = len(off) - 1
        off = np.ascontiguousarray(off, dtype=np.uint64)
        ts_in = np.ascontiguousarray(ts, dtype=np.int64)
        C_ = len(self.cols)
        if alloc is None:
            def alloc(nb):
                a = np.empty(max(1, nb), np.uint8)
                return a, a
        owners = []

        def take(nb, dtype):
            a, own = alloc(nb * np.dtype(dtype).itemsize)
            owners.append(own)
            return a[: nb * np.dtype(dtype).itemsize].view(dtype)
        frames = -(-max(1, n) // abi.HSG_TS16_FRAME)
        key = take(n, np.uint32)
        tsb = take(n, np.int64)
        fr = take(frames, np.int64)
        cols = [take(n, np.int64) for _ in range(C_)]
        valid = [take(n, np.uint8) for _ in range(C_)]
        cp = (C.c_void_p * max(1, C_))(*[c.ctypes.data for c in cols])
        vp = (C.c_void_p * max(1, C_))(*[v.ctypes.data for v in valid])
        bufs = abi.hsg_decode_buffers(capacity=n, key_id=key.ctypes.data, ts=tsb.ctypes.data, ts_frames=fr.ctypes.data,
                                      cols=C.cast(cp, C.POINTER(C.c_void_p)), valid=C.cast(vp, C.POINTER(C.c_void_p)),
                                      allow=int(allow))
        out = abi.hsg_batch()
        status = np.empty(n, np.uint8)
        rej = C.c_uint64()
        spell = np.empty(n, np.uint32) if spellings else None
        _check(self._L.hsg_decode_json_batch(self._h, keys.handle, n, buf, off.ctypes.data, ts_in.ctypes.data,
                                             C.byref(bufs), C.byref(out), status.ctypes.data, C.byref(rej),
                                             spell.ctypes.data if spellings else None, int(threads)),
               "hsg_decode_json_batch")
        return DecodedBatch(out, bufs, (owners, cp, vp, key, tsb, fr, cols, valid), status, int(rej.value), spell,
                            [t for _, t, _ in self.cols])

    def close(self):
        if self._h:
            self._L.hsg_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DecodedBatch:
    """A decoded poll batch in its transport encoding (hsg_decode_json_batch):
    .batch is the hsg_batch to push (OpHandle.push_batch), the arrays it
    points into are kept alive here."""

    def __init__(self, batch, bufs, keep, status, rejected, spell, col_types):
        self.batch, self._bufs, self._keep = batch, bufs, keep
        self.status, self.rejected, self.spell, self.col_types = status, rejected, spell, col_types

    @property
    def n(self):
        return int(self.batch.n)

    def bytes_per_record(self) -> float:
        """Transport bytes of the batch (what crosses PCIe) per record."""
        b = self.batch
        n = max(1, self.n)
        kb = 2 if b.key_enc == abi.HSG_ENC_K16 else 4
        tb = {abi.HSG_ENC_TS16: 2, abi.HSG_ENC_TS32: 4}.get(b.ts_enc, 8)
        fr = 8 * (-(-self.n // abi.HSG_TS16_FRAME)) / n if b.ts_enc == abi.HSG_ENC_TS16 else 0.0
        cb = sum(4 if b.col_enc[c] != abi.HSG_ENC_FULL else 8 for c in range(b.n_cols))
        vb = sum(1 for c in range(b.n_cols) if self._bufs.valid_ptrs[c])
        return kb + tb + fr + cb + vb

    def widen(self):
        """The batch back at full width on the host (key_id u32, ts i64, cols,
        valid or None per column): what the device's widening produces."""
        b, n = self.batch, self.n
        _owners, _cp, _vp, key, tsb, fr, cols, valid = self._keep
        k = key.view(np.uint16)[:n].astype(np.uint32) if b.key_enc == abi.HSG_ENC_K16 else key[:n].copy()
        if b.ts_enc == abi.HSG_ENC_TS16:
            t = np.repeat(fr[: -(-n // abi.HSG_TS16_FRAME)], abi.HSG_TS16_FRAME)[:n] + tsb.view(np.uint16)[:n]
        elif b.ts_enc == abi.HSG_ENC_TS32:
            t = b.ts_base + tsb.view(np.int32)[:n].astype(np.int64)
        else:
            t = tsb[:n].copy()
        out = []
        for c, ty in enumerate(self.col_types):
            e = b.col_enc[c]
            if e == abi.HSG_ENC_I32:
                out.append(cols[c].view(np.int32)[:n].astype(np.int64))
            elif e == abi.HSG_ENC_DEC32:
                out.append(cols[c].view(np.int32)[:n].astype(np.float64) / 10.0 ** b.col_scale[c])
            else:
                out.append(cols[c][:n].view(np.float64 if ty == abi.HSG_F64 else np.int64).copy())
        vs = [valid[c][:n].copy() if self._bufs.valid_ptrs[c] else None for c in range(len(self.col_types))]
        return k, t, out, vs


def pack_records(values: Sequence[bytes]):
    """Record values -> (buffer, offsets) as hsg_decode_json takes them."""
    lens = np.fromiter((len(v) for v in values), dtype=np.uint64, count=len(values))
    off = np.zeros(len(values) + 1, np.uint64)
    np.cumsum(lens, out=off[1:])
    return b"".join(values), off
