"""GPU parity of the session store's less common paths against the oracle
(SessionWindowedStream.hs:84-118, Store.hs:243-272): hot keys whose bucket
is merged chunk by chunk (k_ss_merge_big), arena compaction / growth in the
middle of a batch (merge and replay paths), key-table growth by rehash."""
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
    e = Engine(device=0, batch_capacity=1 << 20)
    yield e
    e.close()


def _drive(eng, spec, batches, faithful=True):
    g, o = eng.op(spec), pyoracle.OracleOp(spec, faithful_sessions=faithful)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, (key, ts, cols, valid) in enumerate(batches):
        wg = g.push(key, ts, cols, valid, watermark=wg)
        wo = o.push(key, ts, cols, valid, watermark=wo)
        assert wg == wo
        if spec.emit_mode != abi.HSG_EMIT_NONE:
            rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                       what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state")
    st = g.stats()
    g.close()
    o.close()
    return st


def _hot_batches(seed, n, nb=3, hot_frac=0.4):
    out = []
    for bi in range(nb):
        key, ts, cols, valid = gen_small(seed + bi, n, 50_000, col_types=(abi.HSG_I64, abi.HSG_F64),
                                         span=200_000, base=20_000_000 + bi * 150_000)
        rng = np.random.default_rng(seed + 100 + bi)
        hot = rng.random(n) < hot_frac
        key = np.where(hot & (key != abi.HSG_KEY_NONE), rng.integers(0, 3, size=n).astype(np.uint32), key)
        out.append((key.astype(np.uint32), ts, cols, valid))
    return out


@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_NONE], ids=["per_batch", "none"])
@pytest.mark.parametrize("gap", [0, 500, 5_000])
def test_hot_keys_big_buckets(eng, mode, gap):
    """A few keys take 40 % of each batch: their buckets exceed one LDS sort
    and are merged chunk by chunk (k_ss_merge_big), the rest by k_ss_apply."""
    aggs = [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MIN, 1), (abi.HSG_MAX, 0), (abi.HSG_AVG, 1),
            (abi.HSG_COUNT, 1)]
    spec = OpSpec(abi.HSG_SESSION, mode, gap_ms=gap, col_types=[abi.HSG_I64, abi.HSG_F64], aggs=aggs)
    _drive(eng, spec, _hot_batches(11, 300_000), faithful=False)


@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_PER_RECORD], ids=["merge", "replay"])
def test_arena_refill_mid_batch(eng, mode):
    """A 1024-row arena floor: every batch outgrows it, so blocks / chunks that
    cannot reserve their lists stop, the host compacts and grows the arena and
    the batch resumes; the result is unchanged."""
    from hstream_amd.engine import testing_knob
    spec = OpSpec(abi.HSG_SESSION, mode, gap_ms=300, col_types=[abi.HSG_I64, abi.HSG_F64],
                  aggs=ALL_AGG_SETS["mixed"] if mode == abi.HSG_EMIT_PER_RECORD else
                  [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_SUM, 1)], state_capacity=16)
    batches = [gen_small(500 + bi, 40_000, 3_000, col_types=spec.col_types, span=120_000,
                         base=7_000_000 + bi * 100_000) for bi in range(4)]
    batches += _hot_batches(77, 20_000, nb=2)
    with testing_knob(abi.HSG_KNOB_SESS_ARENA_MIN, 1024):
        _drive(eng, spec, batches, faithful=False)


def test_key_table_growth(eng):
    """state_capacity 16: the key table starts at its floor and is rehashed
    as 400K distinct keys arrive over the batches."""
    spec = OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_BATCH, gap_ms=1_000, col_types=[abi.HSG_I64],
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)], state_capacity=16)
    batches = []
    for bi in range(4):
        rng = np.random.default_rng(900 + bi)
        n = 200_000
        key = rng.integers(0, 400_000, size=n).astype(np.uint32)
        ts = (30_000_000 + bi * 40_000 + np.arange(n) // 10 + rng.integers(0, 3_000, size=n)).astype(np.int64)
        batches.append((key, ts, [rng.integers(-1000, 1000, size=n, dtype=np.int64)], None))
    _drive(eng, spec, batches, faithful=False)


@pytest.mark.parametrize("gap", [0, 1_000, 30_000])
def test_mirror_fast_and_slow_keys(eng, gap):
    """COUNT(*)/SUM sessions (the apply kernel specialised on that program,
    the entry's mirror of the last session valid): each batch mixes keys whose
    records come after their last session (planned from the mirror alone, a
    new session or an extension of the last) with keys whose records reach
    back before it (a galloping search of the list, merges of older
    sessions), and keys new to the table; every batch's changelog and the
    final store against the faithful oracle (Store.hs:243-272)."""
    spec = OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_BATCH, gap_ms=gap, col_types=[abi.HSG_I64],
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)])
    rng = np.random.default_rng(71 + gap)
    batches = []
    t0 = 50_000_000
    for bi in range(5):
        n = 40_000
        key = rng.integers(0, 6_000, size=n).astype(np.uint32)
        ts = t0 + bi * 200_000 + rng.integers(0, 200_000, size=n)
        back = rng.random(n) < 0.15  # reach back into earlier batches' sessions
        ts = np.where(back, ts - rng.integers(100_000, 600_000, size=n), ts).astype(np.int64)
        col = rng.integers(-10**6, 10**6, size=n, dtype=np.int64)
        valid = (rng.random(n) >= 0.03).astype(np.uint8)
        batches.append((key, ts, [col], [valid]))
    _drive(eng, spec, batches, faithful=False)


@pytest.mark.parametrize("ncols", [3, 5, 8])
def test_many_columns_merge_path(eng, ncols):
    """Records of 2 + C words for every C up to kMaxCols through the partition,
    the fused per-sub-bucket merge and the hot-key chunks (each record stride
    is its own kernel instantiation), per-batch mode, with absent fields."""
    types = [abi.HSG_I64 if c % 2 == 0 else abi.HSG_F64 for c in range(ncols)]
    aggs = [(abi.HSG_COUNT_ALL, 0)] + [(abi.HSG_SUM if c % 3 else abi.HSG_MAX, c) for c in range(ncols)]
    spec = OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_BATCH, gap_ms=700, col_types=types, aggs=aggs[:8])
    batches = []
    for bi in range(3):
        key, ts, cols, valid = gen_small(900 + bi, 60_000, 4_000, col_types=tuple(types), span=150_000,
                                         base=9_000_000 + bi * 120_000)
        if bi == 2:  # one hot key: its sub-bucket goes to k_ss_merge_big
            key = np.where((np.arange(key.size) % 3 == 0) & (key != abi.HSG_KEY_NONE), np.uint32(7), key)
        batches.append((key.astype(np.uint32), ts, cols, valid))
    _drive(eng, spec, batches, faithful=False)


@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_RECORD, abi.HSG_EMIT_PER_BATCH], ids=["changes", "per_batch_last"])
@pytest.mark.parametrize("gap", [0, 700, 20_000])
def test_bucket_replay(eng, mode, gap):
    """The bucket replay (EMIT CHANGES, LAST): records partitioned by key hash
    with their arrival indices, grouped by key per sub-bucket in LDS, each
    key's records replayed in arrival order (findSessions / merge, Store.hs
    :243-272, SessionWindowedStream.hs:84-118), the changelog written in
    arrival order from the per-record states. Out-of-order records, records
    that merge several sessions, absent fields, HSG_KEY_NONE; per batch with
    a passthrough column (LAST: the session's own record order decides)."""
    aggs = ALL_AGG_SETS["mixed"] if mode == abi.HSG_EMIT_PER_RECORD else \
        [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_LAST, 1), (abi.HSG_MAX, 1)]
    spec = OpSpec(abi.HSG_SESSION, mode, gap_ms=gap, col_types=[abi.HSG_I64, abi.HSG_F64], aggs=aggs)
    batches = [gen_small(610 + bi, 150_000, 20_000, col_types=spec.col_types, span=300_000,
                         base=9_000_000 + bi * 200_000) for bi in range(4)]
    st = _drive(eng, spec, batches, faithful=False)
    assert st["replays"] == 0, st  # no sub-bucket over the LDS capacity: every batch took the bucket replay


@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_RECORD, abi.HSG_EMIT_PER_BATCH], ids=["changes", "per_batch_last"])
def test_bucket_replay_hot_key_falls_back(eng, mode):
    """A key with more records in one batch than a bucket-replay sub-bucket
    holds (kBrCap = 1024): the batch is flagged before any state changes and
    runs on the sort-based replay instead; batches without one go back to
    the bucket replay. Same results either way."""
    aggs = ALL_AGG_SETS["mixed"] if mode == abi.HSG_EMIT_PER_RECORD else \
        [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_LAST, 0)]
    spec = OpSpec(abi.HSG_SESSION, mode, gap_ms=400, col_types=[abi.HSG_I64, abi.HSG_F64], aggs=aggs)
    batches = _hot_batches(31, 60_000, nb=2)
    batches.insert(1, gen_small(700, 60_000, 5_000, col_types=spec.col_types, span=200_000, base=20_100_000))
    st = _drive(eng, spec, batches, faithful=False)
    assert st["replays"] == 2, st
