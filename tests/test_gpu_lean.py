"""GPU parity of the lean one-window path (k_agg_lean.hip) across batch-shape
transitions: the host predicts from the previous batch which kernel variants
to launch (packed layout, changelog written by the apply), and a batch that
turns out otherwise is completed after the fetch. Each batch's changelog and
the final state are compared with the CPU oracle (TimeWindowedStream.hs:86-103
per (key, window) group)."""
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
    e = Engine(device=0, batch_capacity=1 << 22)
    yield e
    e.close()


def _uniform(rng, n, nkeys, t0, span):
    key = rng.integers(0, nkeys, size=n).astype(np.uint32)
    ts = (t0 + np.sort(rng.integers(0, span, size=n))).astype(np.int64)
    return key, ts, [rng.integers(-10**9, 10**9, size=n, dtype=np.int64)]


def _batches(seed):
    """uniform (direct changelog) -> hot key (a bucket split over workgroups:
    touched list) -> a span of > 2^16 windows (wide layout) -> uniform ->
    many fresh groups at once (LDS overflow partials) -> uniform."""
    rng = np.random.default_rng(seed)
    out = []
    t = 10_000_000
    out.append(_uniform(rng, 300_000, 2_000, t, 600_000))
    t += 600_000
    k, ts, c = _uniform(rng, 200_000, 2_000, t, 600_000)
    k[rng.random(len(k)) < 0.8] = 7  # ~160K records of one key: its bucket exceeds a workgroup's chunk
    out.append((k, ts, c))
    t += 600_000
    out.append(_uniform(rng, 100_000, 500, t, 2_000_000_000))  # 10 s windows over 23 days
    t += 2_000_000_000
    out.append(_uniform(rng, 300_000, 2_000, t, 600_000))
    t += 600_000
    out.append(_uniform(rng, 400_000, 400_000, t, 6_000_000))  # ~10x the groups the sizing expects
    t += 6_000_000
    out.append(_uniform(rng, 300_000, 2_000, t, 600_000))
    return out


@pytest.mark.parametrize("aggs", [datagen.C_AGGS_FULL, [(abi.HSG_SUM, 0), (abi.HSG_MAX, 0)]],
                         ids=["count_sum_avg_min_max", "sum_max"])
def test_lean_shape_transitions(eng, aggs):
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[abi.HSG_I64], aggs=aggs,
                  state_capacity=1 << 20)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, (key, ts, cols) in enumerate(_batches(5)):
        wg = g.push(key, ts, cols, None, watermark=wg)
        wo = o.push(key, ts, cols, None, watermark=wo)
        assert wg == wo, f"batch {bi}: watermark {wg} != {wo}"
        rows_equal(g.drain(), o.drain(), f64, what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    st = g.stats()
    # the transitions took the paths they are meant to: lean batches, direct
    # changelogs, and replays of the emit chain (the hot-key and the
    # overflowing batch, each after a direct one)
    assert st["lean_batches"] >= 4 and st["direct_batches"] >= 2, st
    assert st["replays"] >= 1, st
    g.close()
    o.close()


def test_lean_late_batch_after_prediction(eng):
    """A batch with records beyond the grace (careful path) between lean
    batches: the prediction must not skip kernels the careful path needs."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[abi.HSG_I64],
                  aggs=datagen.C_AGGS_FULL, state_capacity=1 << 20)
    rng = np.random.default_rng(9)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    wg = wo = -1
    t = 50_000_000
    for bi in range(5):
        key, ts, cols = _uniform(rng, 200_000, 3_000, t, 300_000)
        if bi == 3:
            ts[::50] -= abi.HSG_DEFAULT_GRACE_MS + 400_000  # late by more than the grace
        t += 300_000
        wg = g.push(key, ts, cols, None, watermark=wg)
        wo = o.push(key, ts, cols, None, watermark=wo)
        assert wg == wo
        rows_equal(g.drain(), o.drain(), spec.agg_is_f64(), what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), spec.agg_is_f64(), what="state dump")
    g.close()
    o.close()


@pytest.mark.parametrize("ctype", [abi.HSG_I64, abi.HSG_F64], ids=["i64", "f64"])
def test_lean_later_batch_with_identity_partials(eng, ctype):
    """A group's later batch whose partial equals the slot identities (its
    values cancel to a zero SUM, or every record lacks the field): the row
    keeps its earlier state (Codegen.hs:423-461: an absent field leaves the
    accumulator alone, +0 changes nothing)."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[ctype],
                  aggs=datagen.C_AGGS_FULL, state_capacity=1 << 20)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    dt = np.float64 if ctype == abi.HSG_F64 else np.int64
    n = 4096
    key = np.arange(n, dtype=np.uint32) % 512
    ts = np.full(n, 1_000_000, np.int64) + np.arange(n)
    v1 = (np.arange(n) % 97 - 40).astype(dt)
    # second batch: keys 0..255 get +x, -x pairs (partial SUM 0), keys 256..511 only absent fields
    key2 = np.concatenate([np.repeat(np.arange(256, dtype=np.uint32), 8), np.arange(256, 512, dtype=np.uint32)])
    v2 = np.concatenate([np.tile(np.array([7, -7], dt), 1024), np.zeros(256, dt)])
    valid2 = np.concatenate([np.ones(2048, np.uint8), np.zeros(256, np.uint8)])
    ts2 = np.full(key2.size, 1_005_000, np.int64)
    wg = g.push(key, ts, [v1], None, watermark=-1)
    wo = o.push(key, ts, [v1], None, watermark=-1)
    rows_equal(g.drain(), o.drain(), spec.agg_is_f64(), what="batch 0")
    wg = g.push(key2, ts2, [v2], [valid2], watermark=wg)
    wo = o.push(key2, ts2, [v2], [valid2], watermark=wo)
    assert wg == wo
    rows_equal(g.drain(), o.drain(), spec.agg_is_f64(), what="batch 1")
    rows_equal(g.dump_state(), o.dump_state(), spec.agg_is_f64(), what="state dump")
    g.close()
    o.close()


def test_table_room_holds_and_regrows(eng):
    """The table is sized for twice the last lean batch's groups, not one group
    per record: a batch with more new groups than the room left holds back
    before claiming (the lean apply on its partials, the general kernels on
    the worst case of a wide batch), and runs again on a grown table. Starts
    from a 2048-slot table so every kind of hold happens; each changelog and
    the final state match the oracle."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[abi.HSG_I64],
                  aggs=datagen.C_AGGS_FULL, state_capacity=1 << 10)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    rng = np.random.default_rng(11)
    t = 10_000_000
    batches = []
    # (a region filled by a few keys with many windows spills into the
    # overflow rows: test_gpu_regions.py)
    for nkeys, span, n in [(20_000, 600_000, 300_000),        # ~260K groups >> 1.5K room: lean hold
                           (20_000, 600_000, 300_000),        # inside the prediction
                           (5_000, 2_000_000_000, 100_000),   # > 2^16 windows: wide layout
                           (20_000, 600_000, 300_000),
                           (300_000, 600_000, 400_000),       # ~1.5x the predicted groups: lean hold
                           (20_000, 600_000, 300_000)]:
        batches.append(_uniform(rng, n, nkeys, t, span))
        t += span
    wg = wo = -1
    for bi, (key, ts, cols) in enumerate(batches):
        wg = g.push(key, ts, cols, None, watermark=wg)
        wo = o.push(key, ts, cols, None, watermark=wo)
        assert wg == wo, f"batch {bi}: watermark {wg} != {wo}"
        rows_equal(g.drain(), o.drain(), f64, what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    st = g.stats()
    assert st["grow_events"] >= 2 and st["replays"] >= 2, st
    g.close()
    o.close()


def test_table_sized_by_groups_not_records(eng):
    """A steady one-window stream (C2's shape: few groups per record) keeps a
    table sized by its groups: 2^22-record batches over 4K keys (~45K groups
    per batch) keep the engine's default 4M-slot table, where one new group
    per record would grow it to 8M slots on the first batch."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=60_000, col_types=[abi.HSG_I64],
                  aggs=datagen.C_AGGS_FULL)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    rng = np.random.default_rng(12)
    t = 0
    wg = wo = -1
    for bi in range(3):
        key, ts, cols = _uniform(rng, 1 << 22, 4_096, t, 600_000)
        t += 600_000
        wg = g.push(key, ts, cols, None, watermark=wg)
        wo = o.push(key, ts, cols, None, watermark=wo)
        rows_equal(g.drain(), o.drain(), f64, what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    st = g.stats()
    assert st["table_slots"] <= (1 << 22) and st["grow_events"] == 0, st
    g.close()
    o.close()


@pytest.mark.parametrize("hot", [False, True], ids=["uniform", "hot_key"])
def test_hopping_deferred_hold_across_rebuild(eng, hot):
    """Hopping per-batch changelog when k_seg_apply holds its deferred window
    updates back for table room: the table is rebuilt in the middle of the
    batch (after k_part_agg's own updates went in), so the touched-list
    entries k_part_agg made -- slots of the old table -- must follow their
    groups into the new one. The table is sized from the last batch's
    deferred updates, so a batch with several times the previous batch's new
    groups holds; a hot key splits its bucket over workgroups, whose
    in-kernel updates fill the touched list before the hold. Every changelog
    and the final state match the oracle (TimeWindowedStream.hs:86-103)."""
    spec = OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_BATCH, size_ms=60_000, advance_ms=5_000,
                  col_types=[abi.HSG_I64], aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MAX, 0)])
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    rng = np.random.default_rng(23 + hot)
    t = 10_000_000
    wg = wo = -1
    for bi, (nkeys, span, n) in enumerate([(2_000, 120_000, 200_000),     # ~48K groups
                                           (2_000, 120_000, 200_000),
                                           (400_000, 600_000, 1_000_000),  # several times the room predicted
                                           (2_000, 120_000, 200_000),
                                           (1_000_000, 1_200_000, 2_000_000)]):
        key, ts, cols = _uniform(rng, n, nkeys, t, span)
        if hot and bi >= 2:
            key[rng.random(n) < 0.3] = 11
        t += span
        wg = g.push(key, ts, cols, None, watermark=wg)
        wo = o.push(key, ts, cols, None, watermark=wo)
        assert wg == wo, f"batch {bi}: watermark {wg} != {wo}"
        rows_equal(g.drain(), o.drain(), f64, what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    st = g.stats()
    assert st["grow_events"] >= 1 and st["replays"] >= 1, st
    g.close()
    o.close()
