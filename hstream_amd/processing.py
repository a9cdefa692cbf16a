"""Host-side mirror of the reference's Stream DSL for the windowed GROUP BY path.

Names and argument meaning follow hstream-processing (Yu-zh/hstream):

  TimeWindows / mkTumblingWindow / mkHoppingWindow   Stream/TimeWindows.hs:23-43
  TimeWindow / TimeWindowKey                         Stream/TimeWindows.hs:45-63
  SessionWindows / mkSessionWindows                  Stream/SessionWindows.hs:20-30
  GroupedStream.timeWindowedBy / sessionWindowedBy   Stream/GroupedStream.hs:89-117
  GroupedStream / TimeWindowedStream / SessionWindowedStream .aggregate / .count
                                                     GroupedStream.hs:35-69,
                                                     TimeWindowedStream.hs:32-70,
                                                     SessionWindowedStream.hs:33-72
  Materialized                                       Stream/Internal.hs:123-128
  runTask (poll loop + stream time)                  Processor.hs:99-144
  time-window / session key serdes                   TimeWindows.hs:68-93,
                                                     hstream-sql/.../Codegen/Boilerplate.hs:60-88

The reference processes one record at a time through a topology; here an
operator is one libhstream_gpu op and a poll batch is handed over whole.
Records arrive as (key, value-object, timestamp) like SourceRecord
(Type.hs), the group key is dictionary-encoded to a u32 id with the
reference's key equality (Aeson values: 1 and 1.0 are one key), and the
aggregated fields are extracted into typed columns. A record whose
aggregated field has the wrong type makes the reference throw before any
window is updated (Codegen.hs:430-431, Processor.hs:140-143); it is passed as
HSG_KEY_NONE so it still moves stream time, exactly like a record the WHERE
clause filtered.
"""
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .columnar import OpSpec, Rows

GRACE_MS = abi.HSG_DEFAULT_GRACE_MS  # 24 * 3600 * 1000


# ---------------------------------------------------------------------------
# window specs (Stream/TimeWindows.hs, Stream/SessionWindows.hs)
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class TimeWindows:
    twSizeMs: int
    twAdvanceMs: int
    twGraceMs: int = GRACE_MS


def mkTumblingWindow(windowSize: int) -> TimeWindows:
    return TimeWindows(windowSize, windowSize, GRACE_MS)


def mkHoppingWindow(windowSize: int, stepSize: int) -> TimeWindows:
    return TimeWindows(windowSize, stepSize, GRACE_MS)


@dataclass(frozen=True)
class SessionWindows:
    swInactivityGap: int
    swGraceMs: int = GRACE_MS  # defined by the reference, never read


def mkSessionWindows(inactivityGap: int) -> SessionWindows:
    return SessionWindows(inactivityGap, GRACE_MS)


@dataclass(frozen=True, order=True)
class TimeWindow:
    tWindowStart: int
    tWindowEnd: int


@dataclass(frozen=True)
class TimeWindowKey:
    twkKey: Any
    twkWindow: TimeWindow


# ---------------------------------------------------------------------------
# key and window serdes at the output boundary
# ---------------------------------------------------------------------------
def time_window_bytes(w: TimeWindow) -> bytes:
    """timeWindowSerde: int64BE start ++ int64BE 0 (Boilerplate.hs:60-74)."""
    return struct.pack(">qq", w.tWindowStart, 0)


def session_window_bytes(w: TimeWindow) -> bytes:
    """sessionWindowSerde: int64BE start ++ int64BE end (Boilerplate.hs:76-88)."""
    return struct.pack(">qq", w.tWindowStart, w.tWindowEnd)


def time_window_key_bytes(key_bytes: bytes, w: TimeWindow, session=False) -> bytes:
    """timeWindowKeySerializer: compose (window bytes, key bytes) (TimeWindows.hs:68-73)."""
    return (session_window_bytes(w) if session else time_window_bytes(w)) + key_bytes


def time_window_key_from_bytes(b: bytes, window_size: int, session=False) -> Tuple[bytes, TimeWindow]:
    """timeWindowKeyDeserializer: split at 16, end = start + size (TimeWindows.hs:75-85)."""
    start, second = struct.unpack(">qq", b[:16])
    end = second if session else start + window_size
    return b[16:], TimeWindow(start, end)


# ---------------------------------------------------------------------------
# key dictionary with the reference's key equality
# ---------------------------------------------------------------------------
def _canon(v):
    # Aeson Number is Scientific: 1 == 1.0; bools are not numbers
    if isinstance(v, bool) or v is None:
        return ("b", v)
    if isinstance(v, (int, float, np.integer, np.floating)):
        f = float(v)
        if f.is_integer():
            return ("n", int(f))
        return ("n", f)
    if isinstance(v, dict):
        return ("o", tuple(sorted((k, _canon(x)) for k, x in v.items())))
    if isinstance(v, (list, tuple)):
        return ("a", tuple(_canon(x) for x in v))
    return ("s", v)


class KeyDict:
    """Group key <-> u32 id. HSG_KEY_NONE is never handed out."""

    def __init__(self):
        self._ids: Dict[Any, int] = {}
        self._keys: List[Any] = []

    def encode(self, key) -> int:
        c = _canon(key)
        i = self._ids.get(c)
        if i is None:
            i = len(self._keys)
            if i >= abi.HSG_KEY_NONE:
                raise OverflowError("key dictionary full")
            self._ids[c] = i
            self._keys.append(key)
        return i

    def decode(self, i: int):
        return self._keys[int(i)]

    def __len__(self):
        return len(self._keys)


# ---------------------------------------------------------------------------
# aggregates: the SQL components the codegen builds (Codegen.hs:399-469)
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class Agg:
    kind: int                 # abi.HSG_COUNT_ALL ...
    field: Optional[str] = None
    alias: Optional[str] = None
    is_float: bool = False    # the column's type (numbers with decimals -> f64)

    @property
    def name(self):
        if self.alias:
            return self.alias
        n = {abi.HSG_COUNT_ALL: "COUNT(*)", abi.HSG_COUNT: "COUNT", abi.HSG_SUM: "SUM", abi.HSG_MIN: "MIN",
             abi.HSG_MAX: "MAX", abi.HSG_AVG: "AVG", abi.HSG_LAST: ""}[self.kind]
        return n if self.kind == abi.HSG_COUNT_ALL else (f"{n}({self.field})" if n else self.field)


def COUNT_ALL(alias=None):
    return Agg(abi.HSG_COUNT_ALL, None, alias)


def COUNT(f, alias=None):
    return Agg(abi.HSG_COUNT, f, alias)


def SUM(f, alias=None, is_float=False):
    return Agg(abi.HSG_SUM, f, alias, is_float)


def MIN(f, alias=None, is_float=False):
    return Agg(abi.HSG_MIN, f, alias, is_float)


def MAX(f, alias=None, is_float=False):
    return Agg(abi.HSG_MAX, f, alias, is_float)


def AVG(f, alias=None, is_float=False):
    return Agg(abi.HSG_AVG, f, alias, is_float)


def LAST(f, alias=None, is_float=False):
    """A non-aggregate SELECT column: the last record's value (Codegen.hs:463-469)."""
    return Agg(abi.HSG_LAST, f, alias, is_float)


@dataclass
class Materialized:
    """mKeySerde/mValueSerde/mStateStore (Stream/Internal.hs:123-128): the key
    dictionary plays the key serde, the HBM table the state store."""

    keys: KeyDict = field(default_factory=KeyDict)
    state_capacity: int = 0
    out_capacity: int = 0


# ---------------------------------------------------------------------------
# streams and tables
# ---------------------------------------------------------------------------
class GroupedStream:
    """A re-keyed stream (Stream.groupBy, Stream.hs:196-211)."""

    def __init__(self, engine, key_field: str):
        self.engine = engine
        self.key_field = key_field

    def timeWindowedBy(self, windows: TimeWindows) -> "TimeWindowedStream":
        return TimeWindowedStream(self, windows)

    def sessionWindowedBy(self, windows: SessionWindows) -> "SessionWindowedStream":
        return SessionWindowedStream(self, windows)

    def aggregate(self, aggs: Sequence[Agg], materialized: Materialized, emit=abi.HSG_EMIT_PER_RECORD) -> "Table":
        return Table(self, OpSpec(abi.HSG_UNWINDOWED, emit), aggs, materialized)

    def count(self, materialized: Materialized, emit=abi.HSG_EMIT_PER_RECORD) -> "Table":
        return self.aggregate([COUNT_ALL("count")], materialized, emit)


def groupBy(engine, key_field: str) -> GroupedStream:
    return GroupedStream(engine, key_field)


class TimeWindowedStream:
    def __init__(self, grouped: GroupedStream, windows: TimeWindows):
        self.grouped = grouped
        self.windows = windows

    def aggregate(self, aggs, materialized, emit=abi.HSG_EMIT_PER_RECORD) -> "Table":
        w = self.windows
        kind = abi.HSG_TUMBLING if w.twAdvanceMs == w.twSizeMs else abi.HSG_HOPPING
        spec = OpSpec(kind, emit, size_ms=w.twSizeMs, advance_ms=w.twAdvanceMs, grace_ms=w.twGraceMs)
        return Table(self.grouped, spec, aggs, materialized)

    def count(self, materialized, emit=abi.HSG_EMIT_PER_RECORD) -> "Table":
        return self.aggregate([COUNT_ALL("count")], materialized, emit)


class SessionWindowedStream:
    def __init__(self, grouped: GroupedStream, windows: SessionWindows):
        self.grouped = grouped
        self.windows = windows

    def aggregate(self, aggs, materialized, emit=abi.HSG_EMIT_PER_RECORD) -> "Table":
        spec = OpSpec(abi.HSG_SESSION, emit, gap_ms=self.windows.swInactivityGap)
        return Table(self.grouped, spec, aggs, materialized)

    def count(self, materialized, emit=abi.HSG_EMIT_PER_RECORD) -> "Table":
        return self.aggregate([COUNT_ALL("count")], materialized, emit)


class Table:
    """The aggregate operator's output table (Table.hs), backed by one GPU op.

    process(records) runs one poll batch; it returns the changelog rows as
    (TimeWindowKey | key, {alias: value}) in the order the reference forwards
    them (per-record mode) or one row per touched group (per-batch mode)."""

    def __init__(self, grouped: GroupedStream, spec: OpSpec, aggs: Sequence[Agg], materialized: Materialized):
        self.grouped = grouped
        self.aggs = list(aggs)
        self.mat = materialized
        fields: List[Tuple[str, bool]] = []
        for a in self.aggs:
            if a.kind != abi.HSG_COUNT_ALL and (a.field, a.is_float) not in fields:
                fields.append((a.field, a.is_float))
        self.fields = fields
        col_of = {fk: i for i, fk in enumerate(fields)}
        # a column read only by COUNT(col) counts any present value (Codegen.hs:412-422);
        # SUM / MIN / MAX / AVG / LAST need a Number (Codegen.hs:423-461)
        self.numeric = [any(a.kind not in (abi.HSG_COUNT_ALL, abi.HSG_COUNT) and (a.field, a.is_float) == fk
                            for a in self.aggs) for fk in fields]
        self._decoder = None
        spec.col_types = [abi.HSG_F64 if fl else abi.HSG_I64 for _, fl in fields]
        spec.aggs = [(a.kind, col_of[(a.field, a.is_float)] if a.kind != abi.HSG_COUNT_ALL else 0) for a in self.aggs]
        spec.state_capacity = materialized.state_capacity
        spec.out_capacity = materialized.out_capacity
        self.spec = spec
        self.op = grouped.engine.op(spec)
        self.windowed = spec.window_kind != abi.HSG_UNWINDOWED

    # -- columnar extraction ------------------------------------------------
    def columns(self, records):
        n = len(records)
        keys = np.empty(n, dtype=np.uint32)
        ts = np.empty(n, dtype=np.int64)
        cols = [np.zeros(n, dtype=np.float64 if fl else np.int64) for _, fl in self.fields]
        valid = [np.ones(n, dtype=np.uint8) for _ in self.fields]
        kf = self.grouped.key_field
        for i, rec in enumerate(records):
            value = rec["value"]
            ts[i] = rec["timestamp"]
            ok = kf in value
            for c, (f, fl) in enumerate(self.fields):
                if f not in value:
                    valid[c][i] = 0  # HM.lookup ... Nothing -> the component leaves the acc alone
                    continue
                v = value[f]
                if not self.numeric[c]:
                    continue  # COUNT(col): present is enough, whatever the value
                if isinstance(v, bool) or not isinstance(v, (int, float, np.integer, np.floating)):
                    ok = False  # "Only columns with Int or Number type ..." aborts the record
                    break
                cols[c][i] = float(v) if fl else int(v)
            keys[i] = self.mat.keys.encode(value[kf]) if ok else abi.HSG_KEY_NONE
        return keys, ts, cols, valid

    def _rows(self, rows: Rows):
        out = []
        for i in range(len(rows)):
            key = self.mat.keys.decode(rows.key_id[i])
            vals = {a.name: rows.aggs[j][i].item() for j, a in enumerate(self.aggs)}
            if self.windowed:
                out.append((TimeWindowKey(key, TimeWindow(int(rows.win_start[i]), int(rows.win_end[i]))), vals))
            else:
                out.append((key, vals))
        return out

    def process_json(self, buf: bytes, off, ts, watermark=-1, threads=0):
        """One poll batch of raw JSON record values (SourceRecord srcValue) and
        their timestamps, decoded by the native ingest (include/hstream_ingest.h)
        straight into the op's columns; needs Materialized(keys=ingest.KeyDict())."""
        from . import ingest
        if not isinstance(self.mat.keys, ingest.KeyDict):
            raise TypeError("process_json needs Materialized(keys=hstream_amd.ingest.KeyDict())")
        if self._decoder is None:
            self._decoder = ingest.Decoder(self.grouped.key_field,
                                           [(f, abi.HSG_F64 if fl else abi.HSG_I64, num)
                                            for (f, fl), num in zip(self.fields, self.numeric)])
        keys, ts_out, cols, valid, _, _ = self._decoder.decode(self.mat.keys, buf, off, ts, threads)
        wm = self.op.push(keys, ts_out, cols, valid, watermark=watermark)
        rows = self.op.drain() if self.spec.emit_mode != abi.HSG_EMIT_NONE else None
        return wm, ([] if rows is None else self._rows(rows))

    def process(self, records, watermark=-1):
        keys, ts, cols, valid = self.columns(records)
        wm = self.op.push(keys, ts, cols, valid, watermark=watermark)
        rows = self.op.drain() if self.spec.emit_mode != abi.HSG_EMIT_NONE else None
        return wm, ([] if rows is None else self._rows(rows))

    def dump(self):
        """ksDump / ssDump (views): every live group."""
        return self._rows(self.op.dump_state())

    def close(self):
        self.op.close()


def runTask(poll, table: Table, max_polls=None, sink=None):
    """Processor.hs:99-144 for one windowed aggregate: poll a batch, advance the
    task's stream time over every polled record, run the operator, forward
    the changelog to `sink`. `poll()` returns a list of records or None."""
    wm = -1  # tcTimestamp starts at -1 (Processor/Internal.hs:151)
    polls = 0
    while max_polls is None or polls < max_polls:
        batch = poll()
        if batch is None:
            break
        wm, rows = table.process(batch, watermark=wm)
        if sink is not None:
            for r in rows:
                sink(r)
        polls += 1
    return wm
