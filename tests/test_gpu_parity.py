"""GPU parity: libhstream_gpu (through the C ABI) against the CPU oracle on the
same seeded inputs. Integer aggregates, keys and window bounds bit-exact; f64
SUM/AVG within 1e-6 relative (util.F64_RTOL)."""
import numpy as np
import pytest

import pyoracle
from hstream_amd import abi, datagen
from hstream_amd.columnar import OpSpec, Rows
from util import ALL_AGG_SETS, gen_small, load_kat, rows_equal, run_kat_case

pytestmark = pytest.mark.gpu

KAT = load_kat()


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need cuda:0"
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=1 << 22)
    yield e
    e.close()


def _pair(eng, spec):
    return eng.op(spec), pyoracle.OracleOp(spec)


def _drive(eng, spec, batches, check_rows=True):
    g, o = _pair(eng, spec)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, (key, ts, cols, valid) in enumerate(batches):
        wg = g.push(key, ts, cols, valid, watermark=wg)
        wo = o.push(key, ts, cols, valid, watermark=wo)
        assert wg == wo, f"batch {bi}: watermark {wg} != {wo}"
        if spec.emit_mode != abi.HSG_EMIT_NONE and check_rows:
            rg, ro = g.drain(), o.drain()
            rows_equal(rg, ro, f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD, what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    return g, o


@pytest.mark.parametrize("case", KAT["cases"], ids=lambda c: c["name"])
def test_reference_kat_gpu(eng, case):
    run_kat_case(case, lambda spec: eng.op(spec))


def _time_specs(modes):
    out = []
    for aggname, col_types in (("count", []), ("full_i64", [abi.HSG_I64]), ("mixed", [abi.HSG_I64, abi.HSG_F64])):
        for kind, kw in ((abi.HSG_TUMBLING, dict(size_ms=10_000)),
                         (abi.HSG_HOPPING, dict(size_ms=10_000, advance_ms=3_000)),
                         (abi.HSG_HOPPING, dict(size_ms=60_000, advance_ms=5_000)),
                         (abi.HSG_UNWINDOWED, {})):
            for mode in modes:
                out.append(pytest.param(OpSpec(kind, mode, col_types=col_types, aggs=ALL_AGG_SETS[aggname], **kw),
                                        id=f"{aggname}-k{kind}-s{kw.get('size_ms', 0)}-m{mode}"))
    return out


@pytest.mark.parametrize("spec", _time_specs([abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_NONE, abi.HSG_EMIT_PER_RECORD]))
def test_time_windows_messy_batches(eng, spec):
    ncols = len(spec.col_types)
    batches = []
    for bi in range(3):
        key, ts, cols, valid = gen_small(1000 + bi, 5000, 37, col_types=spec.col_types or (abi.HSG_I64,),
                                         span=100_000, base=10_000_000 + bi * 100_000)
        batches.append((key, ts, cols[:ncols], valid[:ncols]))
    _drive(eng, spec, batches)


@pytest.mark.parametrize("gap", [0, 700, 2_000])
@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_NONE, abi.HSG_EMIT_PER_RECORD])
def test_session_messy_batches(eng, mode, gap):
    """Sessions with passthrough (LAST) columns: a point that merges into
    existing sessions takes the last overlapped session's value
    (aggregateMergeF _ _ o2, Codegen.hs:467; SessionWindowedStream.hs:99-115)."""
    spec = OpSpec(abi.HSG_SESSION, mode, gap_ms=gap, col_types=[abi.HSG_I64, abi.HSG_F64], aggs=ALL_AGG_SETS["mixed"])
    batches = []
    for bi in range(3):
        batches.append(gen_small(3000 + bi, 5000, 37, col_types=spec.col_types, span=100_000,
                                 base=10_000_000 + bi * 60_000))
    _drive(eng, spec, batches)


@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_PER_RECORD])
def test_edge_batches(eng, mode):
    spec = OpSpec(abi.HSG_HOPPING, mode, size_ms=7, advance_ms=3, col_types=[abi.HSG_I64],
                  aggs=ALL_AGG_SETS["full_i64"])
    e = np.array([], dtype=np.int64)
    batches = [
        (np.array([], dtype=np.uint32), e, [e], None),                                  # empty
        (np.full(4, abi.HSG_KEY_NONE, np.uint32), np.array([5, 9, 1, 2]), [np.arange(4)], None),  # only NONE
        (np.zeros(3, np.uint32), np.array([-5, -1, -100]), [np.arange(3)], None),     # only negative ts
        (np.array([0, 1, 0, 1, 2], np.uint32), np.array([10, 13, 12, 0, 6]), [np.array([5, -3, 7, 1, 0])],
         [np.array([1, 1, 0, 1, 1], np.uint8)]),                                        # size % adv != 0
        (np.array([3, 3], np.uint32), np.array([2**31, 11]), [np.array([1, 2])], None),  # jump then late
    ]
    _drive(eng, spec, batches)


def test_grace_boundary(eng):
    """Window [0,10000) of a record is accepted iff stream time < 10000 + grace."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, aggs=[(abi.HSG_COUNT_ALL, 0)])
    g = abi.HSG_DEFAULT_GRACE_MS
    key = np.zeros(4, np.uint32)
    ts = np.array([10_000 + g - 1, 5, 10_000 + g, 6])  # second record accepted, fourth rejected
    _drive(eng, spec, [(key, ts, [], None)])


def test_device_resident_batch(eng):
    import torch
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=60_000, col_types=[abi.HSG_I64],
                  aggs=datagen.C_AGGS_FULL)
    key, ts, cols, valid = gen_small(5, 100_000, 1000, span=600_000)
    g, o = _pair(eng, spec)
    dk = torch.from_numpy(key.view(np.int32)).cuda()
    dt = torch.from_numpy(ts).cuda()
    dc = [torch.from_numpy(c).cuda() for c in cols]
    dv = [torch.from_numpy(v).cuda() for v in valid]
    wg = g.push(dk, dt, dc, dv, watermark=-1)
    wo = o.push(key, ts, cols, valid, watermark=-1)
    assert wg == wo
    rows_equal(g.drain(), o.drain(), spec.agg_is_f64())
    rows_equal(g.dump_state(), o.dump_state(), spec.agg_is_f64())


@pytest.mark.parametrize("name", ["C1", "C2", "C2f", "C3"])
def test_configs_reduced(eng, name):
    """The BASELINE configs' window specs and aggregates at sizes the oracle finishes in seconds."""
    cfg = datagen.CONFIGS[name]
    n = {"C1": 1_000_000, "C2": 2_000_000, "C2f": 1_000_000, "C3": 300_000}[name]
    wpr = -(-cfg.size_ms // cfg.advance_ms) if cfg.window_kind == abi.HSG_HOPPING else 1
    spec = cfg.spec(abi.HSG_EMIT_PER_BATCH, state_capacity=n * wpr)  # bound on the groups
    batches = []
    bsz = min(n, 1 << 20)
    for s in range(0, n, bsz):
        h = datagen.generate(cfg, n=min(bsz, n - s), start=s, total=n)
        batches.append((h["key_id"], h["ts"], h["cols"] if spec.col_types else [], None))
    _drive(eng, spec, batches)


@pytest.mark.parametrize("kind,kw", [(abi.HSG_HOPPING, dict(size_ms=60_000, advance_ms=5_000)),
                                     (abi.HSG_TUMBLING, dict(size_ms=10_000)),
                                     (abi.HSG_HOPPING, dict(size_ms=50_000, advance_ms=15_000))],
                         ids=["hop-pane", "tumbling", "hop-fanout"])
def test_dense_groups_rounds(eng, kind, kw):
    """More panes per bucket than one LDS table holds: the aggregation's
    key-hash rounds (sized from the previous batch) and overflow rounds; the
    fan-out case spills windows straight to the HBM table."""
    spec = OpSpec(kind, abi.HSG_EMIT_PER_BATCH, col_types=[abi.HSG_I64],
                  aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)], state_capacity=1_000_000, **kw)
    batches = []
    for bi in range(2):
        key, ts, cols, valid = gen_small(7000 + bi, 1 << 17, 12_000, span=60_000,
                                         base=50_000_000 + bi * 60_000, very_late=False, none_frac=0.0,
                                         neg_frac=0.0, absent_frac=0.0)
        batches.append((key, ts, cols, None))
    _drive(eng, spec, batches)


def test_registered_changelog_zero_copy(eng):
    """hsg_op_set_changelog: rows land in caller-owned device columns; drain only counts."""
    import ctypes as C
    import torch
    spec = OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_BATCH, size_ms=60_000, advance_ms=5_000,
                  col_types=[abi.HSG_I64], aggs=datagen.C_AGGS_FULL)
    g, o = _pair(eng, spec)
    cap = 1 << 20
    cols = {k: torch.empty(cap, dtype=t, device="cuda") for k, t in
            (("key", torch.int32), ("ws", torch.int64), ("we", torch.int64), ("src", torch.int64))}
    f64 = spec.agg_is_f64()
    aggs = [torch.empty(cap, dtype=torch.float64 if f else torch.int64, device="cuda") for f in f64]
    ap = (C.c_void_p * len(aggs))(*[a.data_ptr() for a in aggs])
    rows = abi.hsg_rows(capacity=cap, mem=abi.HSG_MEM_DEVICE, n_aggs=len(aggs), key_id=cols["key"].data_ptr(),
                        win_start=cols["ws"].data_ptr(), win_end=cols["we"].data_ptr(),
                        src_index=cols["src"].data_ptr(), aggs=C.cast(ap, C.POINTER(C.c_void_p)))
    g.set_changelog(rows)
    wg = wo = -1
    for bi in range(3):
        key, ts, cv, valid = gen_small(300 + bi, 20_000, 500, span=120_000, base=9_000_000 + bi * 120_000)
        wg = g.push(key, ts, cv, valid, watermark=wg)
        wo = o.push(key, ts, cv, valid, watermark=wo)
        assert wg == wo
        n = g.drain_count()
        torch.cuda.synchronize()
        got = Rows(cols["key"][:n].cpu().numpy().view(np.uint32), cols["ws"][:n].cpu().numpy(),
                   cols["we"][:n].cpu().numpy(), cols["src"][:n].cpu().numpy(), [a[:n].cpu().numpy() for a in aggs])
        rows_equal(got, o.drain(), f64, what=f"zero-copy changelog batch {bi}")
    g.set_changelog(None)
    key, ts, cv, valid = gen_small(399, 5000, 500, span=60_000, base=9_400_000)
    assert g.push(key, ts, cv, valid, watermark=wg) == o.push(key, ts, cv, valid, watermark=wo)
    rows_equal(g.drain(), o.drain(), f64, what="own buffer again")


def test_state_table_grows_instead_of_failing(eng):
    """A batch with more groups than the state capacity: the table is rebuilt
    larger before the batch runs (retention.cpp), no HSG_E_OOM, exact counts."""
    spec = OpSpec(abi.HSG_UNWINDOWED, abi.HSG_EMIT_NONE, aggs=[(abi.HSG_COUNT_ALL, 0)], state_capacity=16)
    g = eng.op(spec)
    key = np.arange(1000, dtype=np.uint32)
    g.push(np.concatenate([key, key[:10]]), np.zeros(1010, np.int64), [], None)
    st = g.stats()
    assert st["state_rows"] == 1000 and st["grow_events"] >= 1
    d = g.dump_state()
    cnt = dict(zip(d.key_id.tolist(), d.aggs[0].tolist()))
    assert cnt == {k: (2 if k < 10 else 1) for k in range(1000)}
    g.close()


def test_changelog_must_be_drained(eng):
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=1000, aggs=[(abi.HSG_COUNT_ALL, 0)],
                  out_capacity=10)
    g = eng.op(spec)
    g.push(np.zeros(8, np.uint32), np.arange(8, dtype=np.int64), [], None)
    with pytest.raises(abi.HStreamGpuError) as ei:
        g.push(np.zeros(8, np.uint32), np.arange(8, dtype=np.int64), [], None)
    assert ei.value.status == abi.HSG_E_CAPACITY
    assert len(g.drain()) == 8
    g.push(np.zeros(8, np.uint32), np.arange(8, dtype=np.int64), [], None)


def test_reset_clears_state(eng):
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=1000, aggs=[(abi.HSG_COUNT_ALL, 0)])
    g = eng.op(spec)
    g.push(np.zeros(8, np.uint32), np.arange(8, dtype=np.int64), [], None)
    assert len(g.dump_state()) == 1
    g.reset()
    assert len(g.dump_state()) == 0
    g.push(np.zeros(2, np.uint32), np.arange(2, dtype=np.int64), [], None)
    assert g.dump_state().tuples() == [(0, 0, 1000, (2,))]


def test_window_span_limit_is_reported(eng):
    """Window indices are kept relative to the first batch in 32 bits; a record
    2^32 advances away is refused with HSG_E_RANGE, never silently dropped."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_NONE, size_ms=3, aggs=[(abi.HSG_COUNT_ALL, 0)])
    g = eng.op(spec)
    g.push(np.zeros(1, np.uint32), np.array([10], np.int64), [], None)
    with pytest.raises(abi.HStreamGpuError) as ei:
        g.push(np.zeros(1, np.uint32), np.array([3 * 2**33], np.int64), [], None)
    assert ei.value.status == abi.HSG_E_RANGE


# ---------------------------------------------------------------------------
# the multi-GPU exchange path (owner partition, RCCL all-gather + all-to-all-v,
# unpack, sequence numbers, stream-time carry) driven through a 1-rank
# communicator: every record is exchanged with itself
# ---------------------------------------------------------------------------
@pytest.fixture(scope="module")
def xeng():
    import torch
    assert torch.cuda.is_available()
    from hstream_amd.engine import Engine, comm_unique_id
    e = Engine(device=0, rank=0, nranks=1, comm_id=comm_unique_id(), batch_capacity=1 << 20)
    yield e
    e.close()


def _x_specs():
    out = []
    for kind, kw in ((abi.HSG_TUMBLING, dict(size_ms=10_000)), (abi.HSG_HOPPING, dict(size_ms=10_000, advance_ms=3_000)),
                     (abi.HSG_UNWINDOWED, {}), (abi.HSG_SESSION, dict(gap_ms=2_000))):
        aggs = ALL_AGG_SETS["mixed"]
        for mode in (abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_PER_RECORD, abi.HSG_EMIT_NONE):
            out.append(pytest.param(OpSpec(kind, mode, col_types=[abi.HSG_I64, abi.HSG_F64], aggs=aggs, **kw),
                                    id=f"k{kind}-m{mode}"))
    return out


def _owned_expected(spec, batches, xpart):
    """Records aggregated after the exchange: every keyed record on the classic
    path; on the partition-based paths (fast and sequenced) a time-window op's
    record with ts < 0 has no window and does not travel -- it only moves
    stream time, which the all-gathered maxima carry (exchange.cpp
    push_sharded_seq, k_exchange.hip x_sends)."""
    keyed = sum(int((b[0] != abi.HSG_KEY_NONE).sum()) for b in batches)
    if xpart == "classic" or spec.window_kind in (abi.HSG_SESSION, abi.HSG_UNWINDOWED):
        return {keyed}
    windowed = sum(int(((b[0] != abi.HSG_KEY_NONE) & (b[1] >= 0)).sum()) for b in batches)
    return {keyed, windowed}  # (an op without partition buffers takes the classic path)


@pytest.mark.parametrize("xpart", [None, "2", "classic"], ids=["xpart1", "xpart4", "classic"])
@pytest.mark.parametrize("late", [False, True], ids=["no_late", "late"])
@pytest.mark.parametrize("spec", _x_specs())
def test_exchange_path_single_rank(xeng, spec, late, xpart):
    """xpart4: the fast exchange partitions the single rank's records into 4
    owner regions (testing knob HSG_KNOB_XPART_LOG2 = 2), all sent to rank 0,
    so the multi-owner offsets and scatter run with one GPU; late batches,
    per-record changelogs, LAST and sessions take the sequenced exchange (one
    owner region per rank, its stable scatter: tests/test_gpu_two_ranks.py
    runs two owners); classic: the packed classic exchange
    (HSG_KNOB_X_CLASSIC) for them instead."""
    from hstream_amd.engine import testing_knob
    batches = []
    for bi in range(3):
        key, ts, cols, valid = gen_small(2000 + bi, 4000, 29, col_types=spec.col_types, span=60_000,
                                         base=5_000_000 + bi * 60_000, very_late=late)
        batches.append((key, ts, cols, valid))
    with testing_knob(abi.HSG_KNOB_XPART_LOG2, int(xpart) if xpart and xpart != "classic" else -1), \
            testing_knob(abi.HSG_KNOB_X_CLASSIC, 1 if xpart == "classic" else 0):
        g = xeng.op(spec)
    o = pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, (key, ts, cols, valid) in enumerate(batches):
        wg = g.push(key, ts, cols, valid, watermark=wg)
        wo = o.push(key, ts, cols, valid, watermark=wo)
        assert wg == wo
        if spec.emit_mode != abi.HSG_EMIT_NONE:
            rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                       what=f"batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state")
    st = g.stats()
    assert st["records_owned"] in _owned_expected(spec, batches, xpart)


@pytest.mark.parametrize("xpart", [None, "2", "classic"], ids=["xpart1", "xpart4", "classic"])
@pytest.mark.parametrize("spec", _x_specs())
def test_exchange_path_empty_batch_between(xeng, spec, xpart):
    """An empty batch between non-empty ones through the exchange path: the
    empty slice runs no offsets pipeline, so its owner counts must be zero,
    not the previous batch's (the stale runs were sent again and
    re-aggregated)."""
    from hstream_amd.engine import testing_knob
    batches = []
    for bi in range(3):
        key, ts, cols, valid = gen_small(2100 + bi, 4000, 29, col_types=spec.col_types, span=60_000,
                                         base=5_000_000 + bi * 60_000, very_late=False)
        batches.append((key, ts, cols, valid))
    key, ts, cols, valid = batches[0]
    batches.insert(1, (key[:0], ts[:0], [c[:0] for c in cols], [v[:0] for v in valid]))
    with testing_knob(abi.HSG_KNOB_XPART_LOG2, int(xpart) if xpart and xpart != "classic" else -1), \
            testing_knob(abi.HSG_KNOB_X_CLASSIC, 1 if xpart == "classic" else 0):
        g = xeng.op(spec)
    o = pyoracle.OracleOp(spec)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, (key, ts, cols, valid) in enumerate(batches):
        wg = g.push(key, ts, cols, valid, watermark=wg)
        wo = o.push(key, ts, cols, valid, watermark=wo)
        assert wg == wo
        if spec.emit_mode != abi.HSG_EMIT_NONE:
            rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                       what=f"batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state")
    assert g.stats()["records_owned"] in _owned_expected(spec, batches, xpart)


@pytest.mark.parametrize("kind,kw", [(abi.HSG_TUMBLING, dict(size_ms=10_000)),
                                     (abi.HSG_HOPPING, dict(size_ms=10_000, advance_ms=3_000)),
                                     (abi.HSG_UNWINDOWED, {})], ids=["tumbling", "hopping", "unwindowed"])
@pytest.mark.parametrize("late", [False, True], ids=["in_time", "late"])
def test_per_record_groups_span_chunks(eng, kind, kw, late):
    """EMIT CHANGES (TimeWindowedStream.hs:89-103) where a few keys carry
    whole batches (~66K records each, buckets beyond the key sort: hopping
    takes the chunked path): each group's records span many k_pr_local chunks
    of its bucket, which k_pr_carry applies in arrival order; rows in arrival
    x window order, bit-exact against the oracle (LAST included)."""
    spec = OpSpec(kind, abi.HSG_EMIT_PER_RECORD, col_types=[abi.HSG_I64], aggs=ALL_AGG_SETS["full_i64"], **kw)
    batches = []
    for bi in range(3):
        key, ts, cols, valid = gen_small(77 + bi, 200_000, 3, span=40_000, base=5_000_000 + bi * 40_000,
                                         very_late=late)
        batches.append((key, ts, cols, valid))
    _drive(eng, spec, batches)


@pytest.mark.parametrize("nkeys,span", [(20_000, 400_000), (500, 100_000), (4, 100_000)],
                         ids=["wide_ranges", "long_runs", "hot_buckets"])
@pytest.mark.parametrize("late", [False, True], ids=["in_time", "late"])
def test_per_record_key_replay(eng, nkeys, span, late):
    """EMIT CHANGES of hopping windows on the key-grouped replay (k_pr_keys):
    many keys per bucket, so keys share the sort's 12 hash bits (runs of
    several keys); keys whose windows in a batch span more than one wave
    (wide_ranges: ~80 windows), keys with more than 64 records in a batch
    (long_runs) and buckets beyond the LDS key sort (hot_buckets: ~32K
    records, sorted in global scratch); LAST, absent fields, late and keyless records. Rows in
    arrival x window order and the state against the oracle
    (TimeWindowedStream.hs:89-103)."""
    spec = OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_RECORD, size_ms=60_000, advance_ms=5_000,
                  col_types=[abi.HSG_I64], aggs=ALL_AGG_SETS["full_i64"])
    batches = []
    for bi in range(3):
        batches.append(gen_small(910 + bi, 1 << 17, nkeys, span=span, base=7_000_000 + bi * span, very_late=late))
    _drive(eng, spec, batches)


@pytest.mark.parametrize("name", ["C2", "C2f", "C5", "C3"])
def test_per_record_configs_reduced(eng, name):
    """The per-record changelog on the C2 / C2f / C5 workloads at reduced size
    (2 batches of 2^18 records), ordered rows against the oracle."""
    from hstream_amd import datagen
    cfg = datagen.CONFIGS[name]
    spec = cfg.spec(abi.HSG_EMIT_PER_RECORD)
    n, batch = 1 << 19, 1 << 18
    batches = []
    for s in range(0, n, batch):
        h = datagen.generate(cfg, n=batch, start=s, total=n)
        batches.append((h["key_id"], h["ts"], h["cols"], None))
    _drive(eng, spec, batches)


def test_per_record_table_grows(eng):
    """The per-record changelog with a state table far smaller than the groups:
    the table grows between batches (retention.cpp) and the changelog stays
    exact (the per-record scratch is not sized by the table)."""
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=10_000, col_types=[abi.HSG_I64],
                  aggs=ALL_AGG_SETS["full_i64"], state_capacity=256)
    batches = []
    for bi in range(3):
        key, ts, cols, valid = gen_small(300 + bi, 40_000, 5_000, span=30_000, base=2_000_000 + bi * 30_000,
                                         very_late=False)
        batches.append((key, ts, cols, valid))
    g, o = _drive(eng, spec, batches)
    assert g.stats()["grow_events"] >= 1
    g.close()
    o.close()


@pytest.mark.parametrize("sig", ["c2", "count", "full_i64"])
def test_per_record_bucket_segments(eng, sig):
    """EMIT CHANGES of a one-window op whose buckets hold far more groups than
    the per-bucket LDS table (k_pr_bucket walks them in segments, each
    reloading and writing back its groups' rows) together with hot keys whose
    records fill whole waves (the lane-order folds): rows in arrival order and
    the state against the oracle, for the specialised and the runtime slot
    programs (TimeWindowedStream.hs:89-103)."""
    cols = [] if sig == "count" else [abi.HSG_I64]
    aggs = {"count": [(abi.HSG_COUNT_ALL, 0)], "full_i64": ALL_AGG_SETS["full_i64"],
            "c2": [(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_AVG, 0), (abi.HSG_MIN, 0), (abi.HSG_MAX, 0)]}[sig]
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=5_000, col_types=cols, aggs=aggs)
    rng = np.random.default_rng(5)
    batches = []
    for bi in range(3):
        n = 1 << 18
        key = rng.integers(0, 200_000, size=n).astype(np.uint32)
        hot = rng.random(n) < 0.2
        key = np.where(hot, rng.integers(0, 4, size=n), key).astype(np.uint32)
        ts = (80_000_000 + bi * 20_000 + (np.arange(n) * 20_000) // n + rng.integers(0, 1_500, size=n)).astype(np.int64)
        vals = [rng.integers(-10**9, 10**9, size=n, dtype=np.int64) if t == abi.HSG_I64
                else np.round(rng.uniform(-1e6, 1e6, size=n), 3) for t in cols]
        valid = [(rng.random(n) >= 0.05).astype(np.uint8) for _ in cols]
        batches.append((key, ts, vals, valid if cols else None))
    _drive(eng, spec, batches)

