"""GPU parity when a key-hash region of the state table fills while the table
as a whole is moderately loaded.

A key's windows share its region of the HBM table (hsg_tw.h), so a few keys
with many open windows each, or a region that drew more than its share of
keys, can fill one region's sub-table long before the table reaches the load
its growth rule watches. The reference's store never refuses a row
(ksPut = Map.insert, hstream-processing/src/HStream/Processing/Store.hs:66-68):
such groups go to the table's overflow rows, and the next batch rebuilds the
table with larger regions. Every changelog and the final state are compared
with the CPU oracle (TimeWindowedStream.hs:86-103)."""
import dataclasses

import numpy as np
import pytest

import pyoracle
from hstream_amd import abi, datagen
from hstream_amd.columnar import OpSpec
from util import rows_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need cuda:0"
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=1 << 20)
    yield e
    e.close()


def _hot_batch(rng, t0, n_hot, hot_windows, size_ms, n_bg, bg_keys):
    """n_hot keys with one record in each of hot_windows consecutive windows,
    plus n_bg background records over bg_keys keys in the batch's first
    window; arrival order shuffled inside the batch (ts are all within the
    grace, so the order changes no result)."""
    hot = np.repeat(np.arange(n_hot, dtype=np.uint32) + 1_000_000, hot_windows)
    hts = t0 + np.tile(np.arange(hot_windows, dtype=np.int64) * size_ms, n_hot) + rng.integers(0, size_ms, hot.size)
    bg = rng.integers(0, bg_keys, n_bg).astype(np.uint32)
    bts = t0 + rng.integers(0, size_ms, n_bg).astype(np.int64)
    key = np.concatenate([hot, bg])
    ts = np.concatenate([hts, bts]).astype(np.int64)
    perm = rng.permutation(key.size)
    val = rng.integers(-10**6, 10**6, key.size, dtype=np.int64)
    return key[perm], ts[perm], [val]


@pytest.mark.parametrize("emit", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_PER_RECORD, abi.HSG_EMIT_NONE],
                         ids=["per_batch", "per_record", "state_only"])
@pytest.mark.parametrize("kind", [abi.HSG_TUMBLING, abi.HSG_HOPPING], ids=["tumbling", "hopping"])
def test_hot_keys_fill_their_region(eng, emit, kind):
    """Three keys with 6000 open windows each (750 per sub-table of a
    4096-slot region, which holds 512) beside 8000 one-window keys: the table
    stays far below 3/4 load, the hot keys' regions overflow; two more batches
    add 6000 windows per hot key each, so the first rebuild's regions overflow
    again."""
    size = 1_000
    kw = dict(size_ms=size) if kind == abi.HSG_TUMBLING else dict(size_ms=4 * size, advance_ms=size)
    spec = OpSpec(kind, emit, col_types=[abi.HSG_I64], state_capacity=1 << 15,
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MIN, 0), (abi.HSG_MAX, 0)], **kw)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    rng = np.random.default_rng(41)
    wg = wo = -1
    t = 5_000_000
    for bi in range(3):
        key, ts, cols = _hot_batch(rng, t, 3, 6_000, size, 8_000, 8_000)
        t += 6_000 * size
        wg = g.push(key, ts, cols, None, watermark=wg)
        wo = o.push(key, ts, cols, None, watermark=wo)
        assert wg == wo, f"batch {bi}: watermark {wg} != {wo}"
        if emit != abi.HSG_EMIT_NONE:
            rows_equal(g.drain(), o.drain(), f64, ordered=emit == abi.HSG_EMIT_PER_RECORD,
                       what=f"changelog batch {bi}")
        rows_equal(g.dump_state(), o.dump_state(), f64, what=f"state after batch {bi}")
    st = g.stats()
    assert st["overflow_rebuilds"] >= 1, st
    g.close()
    o.close()


def test_c2_stream_over_three_hours(eng):
    """C2's generator (tumbling 60 s, COUNT/SUM/AVG/MIN/MAX, uniform keys,
    near-sorted ts) run over 3 h of event time at 8192 keys: ~1.5M groups in
    an engine-sized table that grows by load in 2^20-record batches; at the
    table's final size a region carries ~16 keys x 180 windows, the fullest
    more than its 4096 slots, while the table is below 3/4 load."""
    cfg = dataclasses.replace(datagen.CONFIGS["C2"], keys=8192, n=6 << 20, span_ms=3 * datagen.HOUR,
                              batch=1 << 20)
    spec = cfg.spec(abi.HSG_EMIT_PER_BATCH)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for s in range(0, cfg.n, cfg.batch):
        h = datagen.generate(cfg, n=cfg.batch, start=s, total=cfg.n)
        wg = g.push(h["key_id"], h["ts"], h["cols"], None, watermark=wg)
        wo = o.push(h["key_id"], h["ts"], h["cols"], None, watermark=wo)
        assert wg == wo
        rows_equal(g.drain(), o.drain(), f64, what=f"changelog at record {s}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    g.close()
    o.close()
