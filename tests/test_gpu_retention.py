"""Retention of the time-window table (hstream_amd/csrc/retention.cpp).

The reference's window store keeps every (key, window) forever and views read
all of it back (TimeWindowedStream.hs:96-100, Store.hs:81,
hstream/src/HStream/Server/Handler.hs:273-315). The ops here start with a state
capacity far below the groups the stream creates: before a batch that could
fill the HBM table the op moves closed windows (end + grace <= stream time) to
host memory and rebuilds the table larger when the open ones need it. Every
push must succeed, every changelog and the final dump (HBM rows + spilled
rows) must equal the oracle's, and the stats must show that spills and
growth happened.
"""
import numpy as np
import pytest

import pyoracle
from hstream_amd import abi
from hstream_amd.columnar import OpSpec
from util import ALL_AGG_SETS, gen_small, rows_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need cuda:0"
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=1 << 18)
    yield e
    e.close()


def _stream(seed, nb, n, nkeys, span, col_types=(abi.HSG_I64,)):
    """nb batches whose time advances by `span` per batch (so older windows
    close as the stream moves on)."""
    out = []
    for b in range(nb):
        key, ts, cols, valid = gen_small(seed + b, n, nkeys, col_types=col_types, span=span,
                                         base=5_000_000 + b * span, late_frac=0.01)
        out.append((key, ts, cols[:len(col_types)], valid[:len(col_types)]))
    return out


def _run_both(eng, spec, batches, wms=None):
    g = eng.op(spec)
    o = pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, (key, ts, cols, valid) in enumerate(batches):
        if wms is not None and wms[bi] is not None:
            wg = wo = wms[bi]
        wg = g.push(key, ts, cols, valid, watermark=wg)
        wo = o.push(key, ts, cols, valid, watermark=wo)
        assert wg == wo, f"batch {bi}"
        if spec.emit_mode != abi.HSG_EMIT_NONE:
            rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                       what=f"changelog batch {bi}")
    st = g.stats()
    exp = o.dump_state()
    assert st["state_rows"] == len(exp)
    rows_equal(g.dump_state(), exp, f64, what="state dump (HBM + spilled)")
    g.close()
    o.close()
    return st


@pytest.mark.parametrize("emit", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_NONE], ids=["per_batch", "none"])
def test_tumbling_spills_closed_windows(eng, emit):
    """1 s tumbling windows, grace 2 s, capacity 256 groups; 12 batches of 20 s
    over 500 keys create ~120K groups. Every batch closes the windows of the
    one before, so the table holds only the open ones."""
    spec = OpSpec(abi.HSG_TUMBLING, emit, size_ms=1000, grace_ms=2000, col_types=[abi.HSG_I64],
                  aggs=ALL_AGG_SETS["full_i64"], state_capacity=256)
    st = _run_both(eng, spec, _stream(11, 12, 20_000, 500, 20_000))
    assert st["spilled_rows"] > 0 and st["spill_events"] > 0
    assert st["grow_events"] > 0


def test_hopping_per_record_spills_and_grows(eng):
    """Hopping 3 s / 1 s, grace 500 ms, exact per-record changelog (the sort
    path's shadow table is resized with the table), f64 and LAST columns."""
    spec = OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_RECORD, size_ms=3000, advance_ms=1000, grace_ms=500,
                  col_types=[abi.HSG_I64, abi.HSG_F64], aggs=ALL_AGG_SETS["mixed"], state_capacity=128)
    st = _run_both(eng, spec, _stream(21, 8, 8_000, 2000, 10_000, col_types=(abi.HSG_I64, abi.HSG_F64)))
    assert st["spilled_rows"] > 0 and st["grow_events"] > 0


def test_unwindowed_grows(eng):
    """No window ever closes without windows: the table only grows, from 64
    groups to the 20K keys."""
    spec = OpSpec(abi.HSG_UNWINDOWED, abi.HSG_EMIT_PER_BATCH, col_types=[abi.HSG_I64],
                  aggs=ALL_AGG_SETS["full_i64"], state_capacity=64)
    st = _run_both(eng, spec, _stream(31, 5, 30_000, 20_000, 5_000))
    assert st["spilled_rows"] == 0 and st["grow_events"] > 0
    assert st["table_slots"] >= 2 * st["state_rows"]


def test_lowered_watermark_reopens_spilled_windows(eng):
    """A caller that restarts its stream time at -1 after windows were spilled
    (runTask never does) makes old windows accept records again: the op brings
    the spilled rows back before the batch, and the result stays the oracle's."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=1000, grace_ms=1000, col_types=[abi.HSG_I64],
                  aggs=ALL_AGG_SETS["full_i64"], state_capacity=256)
    bs = _stream(41, 6, 10_000, 300, 20_000)
    # last batch: records of the first batch's time range, pushed at stream time -1
    key, ts, cols, valid = gen_small(99, 10_000, 300, span=20_000, base=5_000_000, very_late=False)
    bs.append((key, ts, cols[:1], valid[:1]))
    st = _run_both(eng, spec, bs, wms=[None] * 6 + [-1])
    assert st["spill_events"] > 0


def test_device_dump_with_spilled_rows(eng):
    """hsg_dump_state into device columns: spilled rows land after the HBM
    rows at the right offsets."""
    import ctypes as C
    import torch
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_NONE, size_ms=1000, grace_ms=3000, col_types=[abi.HSG_I64],
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)], state_capacity=512)
    bs = _stream(51, 10, 20_000, 300, 20_000)
    g = eng.op(spec)
    o = pyoracle.OracleOp(spec)
    wg = wo = -1
    for key, ts, cols, valid in bs:
        wg = g.push(key, ts, cols, valid, watermark=wg)
        wo = o.push(key, ts, cols, valid, watermark=wo)
    st = g.stats()
    assert st["spilled_rows"] > 0
    n = st["state_rows"]
    key = torch.empty(n, dtype=torch.int32, device="cuda")
    ws, we, src = (torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(3))
    aggs = [torch.empty(n, dtype=torch.int64, device="cuda") for _ in range(2)]
    ap = (C.c_void_p * 2)(*[a.data_ptr() for a in aggs])
    rows = abi.hsg_rows(capacity=n, mem=abi.HSG_MEM_DEVICE, n_aggs=2, key_id=key.data_ptr(), win_start=ws.data_ptr(),
                        win_end=we.data_ptr(), src_index=src.data_ptr(), aggs=C.cast(ap, C.POINTER(C.c_void_p)))
    got = C.c_uint64(0)
    g._check(g._lib.hsg_dump_state(g._h, C.byref(rows), C.byref(got)), "dump_state")
    assert got.value == n
    exp = o.dump_state()
    from hstream_amd.columnar import Rows
    dev = Rows(key.cpu().numpy().view(np.uint32), ws.cpu().numpy(), we.cpu().numpy(), src.cpu().numpy(),
               [a.cpu().numpy() for a in aggs])
    rows_equal(dev, exp, spec.agg_is_f64(), what="device dump")
    g.close()
    o.close()
