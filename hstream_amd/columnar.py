"""Columnar batch / changelog-row marshalling for the C ABI.

Backend-neutral: ``OpSpec`` describes one windowed GROUP BY operator (what the
reference builds with timeWindowedBy/sessionWindowedBy + aggregate,
hstream-sql/src/HStream/SQL/Codegen.hs:479-521) and ``OpHandle`` drives any
library exporting the hsg_op_* call shapes under some symbol prefix. The
product binding (hstream_amd.engine) uses it over libhstream_gpu; the test
oracle binding (oracle/pyoracle.py) uses it over the CPU restatement.
"""
import ctypes as C
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import abi


@dataclass
class OpSpec:
    window_kind: int
    emit_mode: int = abi.HSG_EMIT_PER_BATCH
    size_ms: int = 0
    advance_ms: int = 0
    gap_ms: int = 0
    grace_ms: int = abi.HSG_DEFAULT_GRACE_MS
    col_types: Sequence[int] = ()
    aggs: Sequence[Tuple[int, int]] = ()  # (hsg_agg_kind, column)
    state_capacity: int = 0
    out_capacity: int = 0
    flags: int = 0  # HSG_OPF_* (abi.HSG_OPF_LITERAL_FORMS)

    @property
    def literal_forms(self) -> bool:
        return bool(self.flags & abi.HSG_OPF_LITERAL_FORMS)

    def agg_is_f64(self) -> List[bool]:
        out = []
        for kind, col in self.aggs:
            ct = self.col_types[col] if kind not in (abi.HSG_COUNT_ALL,) and 0 <= col < len(self.col_types) else abi.HSG_I64
            out.append(abi.agg_output_is_f64(kind, ct))
        return out

    def to_config(self):
        n_cols = len(self.col_types)
        col_arr = (C.c_int32 * max(1, n_cols))(*self.col_types)
        agg_arr = (abi.hsg_agg * max(1, len(self.aggs)))(*[abi.hsg_agg(k, c) for k, c in self.aggs])
        adv = self.advance_ms if self.window_kind == abi.HSG_HOPPING else self.size_ms
        cfg = abi.hsg_op_config(
            window_kind=self.window_kind,
            emit_mode=self.emit_mode,
            size_ms=self.size_ms,
            advance_ms=adv,
            gap_ms=self.gap_ms,
            grace_ms=self.grace_ms,
            n_cols=n_cols,
            n_aggs=len(self.aggs),
            col_types=C.cast(col_arr, C.POINTER(C.c_int32)),
            aggs=C.cast(agg_arr, C.POINTER(abi.hsg_agg)),
            state_capacity=self.state_capacity,
            out_capacity=self.out_capacity,
            flags=self.flags,
        )
        return cfg, (col_arr, agg_arr)


def _is_torch(x):
    return type(x).__module__.startswith("torch")


def _ptr(x):
    if x is None:
        return None
    if _is_torch(x):
        return x.data_ptr()
    return x.ctypes.data


def make_batch(key_id, ts, cols=(), valid=None, mem=None, ts_base=None, col_enc=None, col_scale=None,
               ts_frames=None):
    """Build an hsg_batch over numpy arrays (host) or torch tensors (device).

    Returns (hsg_batch, keepalive). Arrays must be contiguous: key_id uint32 /
    int32, ts int64, cols int64 or float64, valid uint8 (or None = all present).
    Narrow transport (include/hstream_gpu.h hsg_enc): a uint16 key_id = ids sent
    as HSG_ENC_K16 (no HSG_KEY_NONE in the batch); ts_base given = ts holds
    int32 offsets from it (HSG_ENC_TS32); ts_frames given = ts holds uint16
    offsets from the base of each HSG_TS16_FRAME-record frame (HSG_ENC_TS16);
    col_enc[c] HSG_ENC_I32 / HSG_ENC_DEC32 = column c holds int32 values /
    decimal mantissas (col_scale[c] digits).
    """
    if mem is None:
        mem = abi.HSG_MEM_DEVICE if (_is_torch(ts) and ts.is_cuda) else abi.HSG_MEM_HOST
    col_enc = list(col_enc or [abi.HSG_ENC_FULL] * len(cols))
    keep = [key_id, ts]
    if not _is_torch(ts):
        key_id = np.asarray(key_id)
        key_id = np.ascontiguousarray(key_id, dtype=np.uint16 if key_id.dtype == np.uint16 else np.uint32)
        ts = np.ascontiguousarray(ts, dtype=np.int32 if ts_base is not None else
                                  np.uint16 if ts_frames is not None else np.int64)
        if ts_frames is not None:
            ts_frames = np.ascontiguousarray(ts_frames, dtype=np.int64)
        cols = [np.ascontiguousarray(c, dtype=np.int32) if e != abi.HSG_ENC_FULL else np.ascontiguousarray(c)
                for c, e in zip(cols, col_enc)]
        if valid is not None:
            valid = [None if v is None else np.ascontiguousarray(v, dtype=np.uint8) for v in valid]
        keep = [key_id, ts, cols, valid, ts_frames]
    else:
        keep.append(ts_frames)
        keep.append(cols)
        keep.append(valid)
    n = int(ts.shape[0])
    ncols = len(cols)
    col_ptrs = (C.c_void_p * max(1, ncols))(*[_ptr(c) for c in cols])
    keep.append(col_ptrs)
    valid_ptrs = None
    if valid is not None:
        valid_ptrs = (C.c_void_p * max(1, ncols))(*[_ptr(v) for v in valid])
        keep.append(valid_ptrs)
    b = abi.hsg_batch(
        n=n,
        mem=mem,
        n_cols=ncols,
        key_id=_ptr(key_id),
        ts=_ptr(ts),
        cols=C.cast(col_ptrs, C.POINTER(C.c_void_p)),
        valid=C.cast(valid_ptrs, C.POINTER(C.c_void_p)) if valid_ptrs is not None else None,
    )
    if str(key_id.dtype) in ("uint16", "torch.int16", "torch.uint16"):
        b.key_enc = abi.HSG_ENC_K16  # (HSG_ENC_K16: ids < 65536, no HSG_KEY_NONE)
    if ts_base is not None:
        b.ts_enc = abi.HSG_ENC_TS32
        b.ts_base = int(ts_base)
    if ts_frames is not None:
        b.ts_enc = abi.HSG_ENC_TS16
        b.ts_frames = _ptr(ts_frames)
    for c, e in enumerate(col_enc):
        b.col_enc[c] = int(e)
        b.col_scale[c] = int(col_scale[c]) if col_scale else 0
    return b, keep


def narrow_keys(key_id):
    """The key column as uint16 (HSG_ENC_K16) when every id fits and no record
    is HSG_KEY_NONE, else unchanged (uint32)."""
    key_id = np.asarray(key_id, dtype=np.uint32)
    if key_id.size and int(key_id.max()) < 65536:
        return key_id.astype(np.uint16)
    return key_id


def narrow_ts16(ts):
    """ts as HSG_ENC_TS16 (frame of reference): (uint16 offsets, int64 frame
    bases) when every frame of HSG_TS16_FRAME records spans < 65536 ms, else
    None."""
    ts = np.asarray(ts, dtype=np.int64)
    f = abi.HSG_TS16_FRAME
    nf = -(-ts.size // f)
    pad = np.empty(nf * f, np.int64)
    pad[:ts.size] = ts
    pad[ts.size:] = ts[-1] if ts.size else 0
    fr = pad.reshape(nf, f)
    lo = fr.min(axis=1)
    if nf and int((fr.max(axis=1) - lo).max()) >= 65536:
        return None
    off = (pad - np.repeat(lo, f))[:ts.size].astype(np.uint16)
    return off, lo


def narrow_columns(ts, cols, col_types, dec_scale=None, ts16=False):
    """What a producer that saw every value (the decoder) can send narrower:
    ts as uint16 offsets from per-frame bases when ts16 and every frame fits
    (the second result is then the int64 frame bases: make_batch ts_frames),
    else as int32 offsets from the batch's minimum when its span fits (the
    second result is that base: make_batch ts_base); i64 columns as int32 when
    every value fits, f64 columns as int32 decimal mantissas when every value
    is a decimal of at most dec_scale[c] digits that fits (checked exactly:
    m / 10^s must give back the value). Returns (ts_arr, ts_base / frames /
    None, cols, col_enc, col_scale); host numpy arrays."""
    ts = np.asarray(ts, dtype=np.int64)
    ts_base = None
    t16 = narrow_ts16(ts) if ts16 and ts.size else None
    if t16 is not None:
        ts, ts_base = t16
    elif ts.size:
        lo, hi = int(ts.min()), int(ts.max())
        if hi - lo < 2**31:
            ts_base = lo
            ts = (ts - lo).astype(np.int32)
    out, enc, scale = [], [], []
    for j, (c, t) in enumerate(zip(cols, col_types)):
        c = np.asarray(c)
        e, sc = abi.HSG_ENC_FULL, 0
        if t == abi.HSG_I64:
            if c.size == 0 or (int(c.min()) >= -2**31 and int(c.max()) < 2**31):
                c, e = c.astype(np.int32), abi.HSG_ENC_I32
        elif dec_scale and dec_scale[j] is not None:
            s = int(dec_scale[j])
            m = np.rint(c * 10.0**s)
            # lossless means bit-identical: -0.0 == 0.0 numerically, but it
            # would come back as +0.0 (f64 MIN / MAX order them, the SUM's
            # text differs), so the comparison is on the bit patterns
            if c.size == 0 or (np.abs(m).max() < 2**31 and np.array_equal(
                    (m.astype(np.int64) / 10.0**s).view(np.int64), np.asarray(c, np.float64).view(np.int64))):
                c, e, sc = m.astype(np.int32), abi.HSG_ENC_DEC32, s
        out.append(c)
        enc.append(e)
        scale.append(sc)
    return ts, ts_base, out, enc, scale


@dataclass
class Rows:
    """Columnar changelog / state rows (host numpy arrays)."""

    key_id: np.ndarray
    win_start: np.ndarray
    win_end: np.ndarray
    src_index: np.ndarray
    aggs: List[np.ndarray] = field(default_factory=list)
    form: Optional[np.ndarray] = None  # literal forms (hsg_rows.form), ops with HSG_OPF_LITERAL_FORMS

    def __len__(self):
        return int(self.key_id.shape[0])

    def sorted(self, by_src=False):
        """Rows in a canonical order: (src_index, win_start) or (key, win_start, win_end)."""
        if by_src:
            order = np.lexsort((self.win_start, self.src_index))
        else:
            order = np.lexsort((self.win_end, self.win_start, self.key_id))
        return Rows(self.key_id[order], self.win_start[order], self.win_end[order],
                    self.src_index[order], [a[order] for a in self.aggs],
                    self.form[order] if self.form is not None else None)

    def tuples(self):
        out = []
        for i in range(len(self)):
            out.append((int(self.key_id[i]), int(self.win_start[i]), int(self.win_end[i]),
                        tuple(a[i].item() for a in self.aggs)))
        return out


def alloc_rows(n: int, agg_is_f64: Sequence[bool], form: bool = False):
    n = int(n)
    arrs = Rows(
        key_id=np.zeros(n, dtype=np.uint32),
        win_start=np.zeros(n, dtype=np.int64),
        win_end=np.zeros(n, dtype=np.int64),
        src_index=np.zeros(n, dtype=np.int64),
        aggs=[np.zeros(n, dtype=np.float64 if f else np.int64) for f in agg_is_f64],
        form=np.zeros(n, dtype=np.uint32) if form else None,
    )
    agg_ptrs = (C.c_void_p * max(1, len(agg_is_f64)))(*[a.ctypes.data for a in arrs.aggs])
    rows = abi.hsg_rows(
        capacity=n,
        mem=abi.HSG_MEM_HOST,
        n_aggs=len(agg_is_f64),
        key_id=arrs.key_id.ctypes.data,
        win_start=arrs.win_start.ctypes.data,
        win_end=arrs.win_end.ctypes.data,
        src_index=arrs.src_index.ctypes.data,
        aggs=C.cast(agg_ptrs, C.POINTER(C.c_void_p)),
        form=arrs.form.ctypes.data if form else None,
    )
    return rows, arrs, agg_ptrs


def truncate(rows: Rows, n: int) -> Rows:
    return Rows(rows.key_id[:n], rows.win_start[:n], rows.win_end[:n], rows.src_index[:n],
                [a[:n] for a in rows.aggs], rows.form[:n] if rows.form is not None else None)


class OpHandle:
    """Drives one operator through a library exposing <prefix>_push_batch etc."""

    def __init__(self, lib, prefix: str, handle, spec: OpSpec):
        self._lib = lib
        self._p = prefix
        self._h = handle
        self.spec = spec
        self._f64 = spec.agg_is_f64()
        self._forms = spec.literal_forms and prefix == "hsg"  # (the oracle keeps no forms)

    def _fn(self, name):
        return getattr(self._lib, f"{self._p}_{name}")

    def _check(self, rc, what):
        if rc != abi.HSG_OK:
            msg = self._fn("last_error")(self._h)
            msg = msg.decode() if msg else ""
            raise abi.HStreamGpuError(rc, f"{what}: {msg}")

    def push(self, key_id, ts, cols=(), valid=None, watermark=-1, mem=None, **enc) -> int:
        """hsg_push_batch; enc = make_batch's narrow transport (ts_base, col_enc, col_scale)."""
        b, keep = make_batch(key_id, ts, cols, valid, mem, **enc)
        wm = C.c_int64(watermark)
        rc = self._fn("push_batch")(self._h, C.byref(b), C.byref(wm))
        del keep
        self._check(rc, "push_batch")
        return wm.value

    def push_batch(self, batch, watermark=-1) -> int:
        """hsg_push_batch of a ready hsg_batch (e.g. DecodedBatch.batch, in the
        decoder's transport encoding)."""
        wm = C.c_int64(watermark)
        rc = self._fn("push_batch")(self._h, C.byref(batch), C.byref(wm))
        self._check(rc, "push_batch")
        return wm.value

    def pending(self) -> int:
        n = C.c_uint64(0)
        self._check(self._fn("pending_rows")(self._h, C.byref(n)), "pending_rows")
        return n.value

    def drain(self) -> Rows:
        n = self.pending()
        rows, arrs, keep = alloc_rows(n, self._f64, self._forms)
        got = C.c_uint64(0)
        self._check(self._fn("drain")(self._h, C.byref(rows), C.byref(got)), "drain")
        return truncate(arrs, got.value)

    def dump_state(self) -> Rows:
        n = C.c_uint64(0)
        self._check(self._fn("state_rows")(self._h, C.byref(n)), "state_rows")
        rows, arrs, keep = alloc_rows(n.value, self._f64, self._forms)
        got = C.c_uint64(0)
        self._check(self._fn("dump_state")(self._h, C.byref(rows), C.byref(got)), "dump_state")
        return truncate(arrs, got.value)

    def reset(self):
        self._check(self._fn("op_reset")(self._h), "op_reset")

    def close(self):
        if self._h:
            self._fn("op_destroy")(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def declare_op_functions(lib, prefix):
    """Set ctypes signatures for the <prefix>_op functions shared by both libraries."""
    vp = C.c_void_p
    P = C.POINTER
    getattr(lib, f"{prefix}_op_destroy").argtypes = [vp]
    getattr(lib, f"{prefix}_op_destroy").restype = None
    getattr(lib, f"{prefix}_op_reset").argtypes = [vp]
    getattr(lib, f"{prefix}_op_reset").restype = C.c_int
    getattr(lib, f"{prefix}_last_error").argtypes = [vp]
    getattr(lib, f"{prefix}_last_error").restype = C.c_char_p
    getattr(lib, f"{prefix}_push_batch").argtypes = [vp, P(abi.hsg_batch), P(C.c_int64)]
    getattr(lib, f"{prefix}_push_batch").restype = C.c_int
    getattr(lib, f"{prefix}_pending_rows").argtypes = [vp, P(C.c_uint64)]
    getattr(lib, f"{prefix}_pending_rows").restype = C.c_int
    getattr(lib, f"{prefix}_drain").argtypes = [vp, P(abi.hsg_rows), P(C.c_uint64)]
    getattr(lib, f"{prefix}_drain").restype = C.c_int
    getattr(lib, f"{prefix}_state_rows").argtypes = [vp, P(C.c_uint64)]
    getattr(lib, f"{prefix}_state_rows").restype = C.c_int
    getattr(lib, f"{prefix}_dump_state").argtypes = [vp, P(abi.hsg_rows), P(C.c_uint64)]
    getattr(lib, f"{prefix}_dump_state").restype = C.c_int
