"""GPU, two ranks: the real multi-rank C++ exchange (hstream_amd/csrc/
exchange.cpp) -- all-gather of the per-rank facts, stream-time carry,
sequence bases, fast-vs-classic decision, owner partition, all-to-all-v,
per-rank aggregation -- driven by two processes that share cuda:0 over the
host transport (HSG_TRANSPORT_HOST: the same collectives through shared
memory instead of RCCL, which needs one GPU per rank). Each rank pushes its
slice of every global batch; the union of the ranks' changelogs and state
must equal one oracle fed the whole stream (keys shard by hash,
each GPU owns its key range, results equal one GPU fed everything).

tests/test_sharded_gloo.py restates the same protocol in Python on the CPU;
this runs the library itself."""
import os
import uuid

import numpy as np
import pytest

from hstream_amd import abi
from hstream_amd.columnar import OpSpec
from test_sharded_gloo import SPECS, _batches, _close
from util import ALL_AGG_SETS

pytestmark = pytest.mark.gpu

GPU_SPECS = dict(SPECS)
# the per-record changelog on the partitioned pipeline (<= 8 slots, with LAST)
GPU_SPECS["hopping_pr_part"] = OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_RECORD, size_ms=10_000, advance_ms=3_000,
                                      col_types=[abi.HSG_I64, abi.HSG_F64], aggs=ALL_AGG_SETS["full_i64"])
GPU_SPECS["tumbling_pr_part"] = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=10_000,
                                       col_types=[abi.HSG_I64, abi.HSG_F64],
                                       aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MAX, 1)])
# sessions on the merge path (per-batch changelog)
GPU_SPECS["session_merge"] = OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_BATCH, gap_ms=2_000,
                                    col_types=[abi.HSG_I64, abi.HSG_F64],
                                    aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MIN, 1)])


def _rows(spec, r):
    if spec.emit_mode == abi.HSG_EMIT_PER_BATCH:
        r.src_index[:] = -1
    return [(int(r.key_id[i]), int(r.win_start[i]), int(r.win_end[i]), int(r.src_index[i]),
             tuple(a[i].item() for a in r.aggs)) for i in range(len(r))]


def _slices(G, late):
    """the protocol test's batches; "empty": rank 0's slice of the middle batch
    is empty (between non-empty ones: its owner runs must not be the previous
    batch's)"""
    if late != "empty":
        return _batches(G, late)
    out = _batches(G, False)
    key, ts, cols, valid = out[1][0]
    out[1][0] = (key[:0], ts[:0], [c[:0] for c in cols], [v[:0] for v in valid])
    return out


def _gpu_worker(rank, G, name, spec_name, late, q):
    try:
        from hstream_amd.engine import Engine
        eng = Engine(device=0, rank=rank, nranks=G, comm_id=name, batch_capacity=1 << 13,
                     transport=abi.HSG_TRANSPORT_HOST)
        spec = GPU_SPECS[spec_name]
        op = eng.op(spec)
        wm, results = -1, []
        for slices in _slices(G, late):
            key, ts, cols, valid = slices[rank]
            wm = op.push(key, ts, cols, valid, watermark=wm)
            results.append(None if spec.emit_mode == abi.HSG_EMIT_NONE else _rows(spec, op.drain()))
        state = op.dump_state().tuples()
        op.close()
        eng.close()
        q.put((rank, wm, results, state))
    except Exception as e:  # reported to the parent, which fails the test
        q.put((rank, "error", repr(e), None))


def _single(spec_name, G, late):
    import pyoracle
    spec = GPU_SPECS[spec_name]
    op = pyoracle.OracleOp(spec)
    wm, results = -1, []
    for slices in _slices(G, late):
        key = np.concatenate([s[0] for s in slices])
        ts = np.concatenate([s[1] for s in slices])
        cols = [np.concatenate([s[2][c] for s in slices]) for c in range(2)]
        valid = [np.concatenate([s[3][c] for s in slices]) for c in range(2)]
        wm = op.push(key, ts, cols, valid, watermark=wm)
        results.append(None if spec.emit_mode == abi.HSG_EMIT_NONE else _rows(spec, op.drain()))
    return wm, results, op.dump_state().tuples()


@pytest.mark.parametrize("late", [False, True, "empty"], ids=["no_late", "late", "empty_slice"])
@pytest.mark.parametrize("spec_name", list(GPU_SPECS))
def test_two_ranks_equal_single_stream(spec_name, late):
    import multiprocessing as mp
    G = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"hsgt-{os.getpid()}-{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_gpu_worker, args=(r, G, name, spec_name, late, q)) for r in range(G)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=100) for _ in range(G)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [o for o in outs if o[1] == "error"]
    assert not errs, errs
    for p in procs:
        assert p.exitcode == 0
    outs.sort(key=lambda o: o[0])
    wm1, res1, st1 = _single(spec_name, G, late)
    assert all(o[1] == wm1 for o in outs), ([o[1] for o in outs], wm1)
    # union of the ranks' state = the single-stream state, keys disjoint
    keys = [set(k for k, *_ in o[3]) for o in outs]
    assert not (keys[0] & keys[1])
    merged = sorted(outs[0][3] + outs[1][3])
    assert len(merged) == len(st1)
    for a, b in zip(merged, sorted(st1)):
        assert a[:3] == b[:3] and _close(a[3], b[3]), (a, b)
    # changelogs: per-record rows carry the global sequence; merged by (src, start)
    for bi in range(len(res1)):
        if res1[bi] is None:
            continue
        rows = sorted(outs[0][2][bi] + outs[1][2][bi], key=lambda t: (t[3], t[1], t[0], t[2], t[4]))
        ref = sorted(res1[bi], key=lambda t: (t[3], t[1], t[0], t[2], t[4]))
        assert len(rows) == len(ref), (bi, len(rows), len(ref))
        for a, b in zip(rows, ref):
            assert a[:4] == b[:4] and _close(a[4], b[4]), (bi, a, b)


# ---------------------------------------------------------------------------
# the stream-stream join, sharded over two ranks (one GPU, host transport)
# ---------------------------------------------------------------------------
def _join_gen(seed, n, nkeys=40, grid=5, span=40_000):
    rng = np.random.default_rng(seed)
    side = (rng.random(n) < 0.5).astype(np.uint8)
    key = rng.integers(0, nkeys, n).astype(np.uint32)
    key[rng.random(n) < 0.01] = abi.HSG_KEY_NONE
    jk = rng.integers(0, 3, n).astype(np.uint32)
    jk[rng.random(n) < 0.03] = abi.HSG_KEY_NONE
    ts = ((np.arange(n) * span) // n + rng.integers(0, 400, n)) // grid * grid
    ts = ts.astype(np.int64) + 1_700_000_000_000
    # handles name the record globally (the caller's values stay where they are)
    handle = np.arange(n, dtype=np.uint64) + (np.uint64(seed) << np.uint64(32))
    return side, key, jk, ts, handle


JOIN_CASES = {"w100_50": (100, 50, 5), "w0_0": (0, 0, 1), "w250_0": (250, 0, 25)}


def _join_slices(case, G):
    """batches of the stream, each cut into G consecutive rank slices (rank
    order = arrival order); the second batch's slice of rank 0 is empty"""
    before, after, grid = JOIN_CASES[case]
    side, key, jk, ts, h = _join_gen(before * 7 + after + grid, 12_000, grid=grid)
    out = []
    for bi, s0 in enumerate(range(0, len(ts), 3_000)):
        b = [a[s0:s0 + 3_000] for a in (side, key, jk, ts, h)]
        cuts = np.linspace(0, len(b[0]), G + 1).astype(int)
        if bi == 1:
            cuts[1] = 0
        out.append([tuple(a[cuts[r]:cuts[r + 1]] for a in b) for r in range(G)])
    return before, after, out


def _join_worker(rank, G, name, case, q):
    try:
        from hstream_amd.engine import Engine
        from hstream_amd.join import Join
        eng = Engine(device=0, rank=rank, nranks=G, comm_id=name, batch_capacity=1 << 13,
                     transport=abi.HSG_TRANSPORT_HOST)
        before, after, batches = _join_slices(case, G)
        j = Join(eng, before, after, batch_capacity=1 << 12)
        rows = []
        for slices in batches:
            j.push(*slices[rank])
            th, oh, k, t = j.drain()
            rows.append(list(zip(th.tolist(), oh.tolist(), k.tolist(), t.tolist())))
        st = j.state_rows()
        j.close()
        eng.close()
        q.put((rank, rows, st))
    except Exception as e:
        q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("case", list(JOIN_CASES))
def test_two_ranks_join_equal_single_stream(case):
    """Each rank pushes its slice of every poll batch; the slices are
    all-gathered, every rank keeps the whole timestamp set and stores /
    probes the records whose key it owns. The union of the two ranks' rows
    (each rank's in arrival order) is the single-stream join's, and the two
    stores hold the single store's entries between them."""
    import multiprocessing as mp
    import joinref
    G = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"hsgj-{os.getpid()}-{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_join_worker, args=(r, G, name, case, q)) for r in range(G)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=100) for _ in range(G)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [o for o in outs if o[1] == "error"]
    assert not errs, errs
    outs.sort(key=lambda o: o[0])
    before, after, batches = _join_slices(case, G)
    ref = joinref.JoinRef(before, after)
    total = 0
    for bi, slices in enumerate(batches):
        whole = [np.concatenate([s[a] for s in slices]) for a in range(5)]
        exp = ref.push(*whole)
        got = outs[0][1][bi] + outs[1][1][bi]
        assert sorted(got) == sorted(exp), (bi, len(got), len(exp))
        # each rank's rows in the single stream's order
        for r in range(G):
            mine = [x for x in exp if x in set(outs[r][1][bi])]
            assert outs[r][1][bi] == mine, (bi, r)
        total += len(exp)
    assert outs[0][2] + outs[1][2] == ref.state_rows()
    assert total > 0 or JOIN_CASES[case][:2] == (0, 0)


# ---------------------------------------------------------------------------
# literal forms through the exchange: the decimal bits ride the
# sequenced exchange's valid bytes (bit 1) and the classic exchange's packed
# word; the sharded result, forms included, equals one GPU fed the whole
# stream (whose forms tests/test_sink.py and test_gpu_sql_shape.py pin
# against the reference's sequential fold)
# ---------------------------------------------------------------------------
FORM_AGGS = [(abi.HSG_LAST, 0), (abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0), (abi.HSG_MIN, 1), (abi.HSG_MAX, 0),
             (abi.HSG_SUM, 1)]
FORM_SPECS = {
    "tumbling_batch": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000,
                             col_types=[abi.HSG_I64, abi.HSG_F64], aggs=FORM_AGGS, flags=abi.HSG_OPF_LITERAL_FORMS),
    "tumbling_changes": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=10_000,
                               col_types=[abi.HSG_I64, abi.HSG_F64], aggs=FORM_AGGS, flags=abi.HSG_OPF_LITERAL_FORMS),
    "session_batch": OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_BATCH, gap_ms=2_000,
                            col_types=[abi.HSG_I64, abi.HSG_F64], aggs=FORM_AGGS, flags=abi.HSG_OPF_LITERAL_FORMS),
    "session_changes": OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_RECORD, gap_ms=2_000,
                              col_types=[abi.HSG_I64, abi.HSG_F64], aggs=FORM_AGGS, flags=abi.HSG_OPF_LITERAL_FORMS),
}


def _form_slices(G):
    """the protocol batches with decimal literals (valid bit 1) on 1 in 4
    present values and a narrow value range (ties)"""
    rng = np.random.default_rng(77)
    out = []
    for slices in _batches(G, False):
        ns = []
        for key, ts, cols, valid in slices:
            c0 = (cols[0] % 7).astype(np.int64)
            c1 = np.round(cols[1] % 5.0, 1)
            v = [(va | ((rng.random(len(va)) < 0.25) & (va != 0)).astype(np.uint8) << 1).astype(np.uint8)
                 for va in valid]
            ns.append((key, ts, [c0, c1], v))
        out.append(ns)
    return out


def _form_rows(spec, r):
    src = [-1] * len(r) if spec.emit_mode == abi.HSG_EMIT_PER_BATCH else r.src_index.tolist()
    return [(int(r.key_id[i]), int(r.win_start[i]), int(r.win_end[i]), int(src[i]), int(r.form[i]),
             tuple(a[i].item() for a in r.aggs)) for i in range(len(r))]


def _form_worker(rank, G, name, spec_name, classic, q):
    try:
        from hstream_amd.engine import Engine, testing_knob
        eng = Engine(device=0, rank=rank, nranks=G, comm_id=name, batch_capacity=1 << 13,
                     transport=abi.HSG_TRANSPORT_HOST)
        spec = FORM_SPECS[spec_name]
        with testing_knob(abi.HSG_KNOB_X_CLASSIC, 1 if classic else 0):
            op = eng.op(spec)
        wm, results = -1, []
        for slices in _form_slices(G):
            key, ts, cols, valid = slices[rank]
            wm = op.push(key, ts, cols, valid, watermark=wm)
            results.append(_form_rows(spec, op.drain()))
        op.close()
        eng.close()
        q.put((rank, wm, results))
    except Exception as e:
        q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("classic", [False, True], ids=["sequenced", "classic"])
@pytest.mark.parametrize("spec_name", list(FORM_SPECS))
def test_two_ranks_literal_forms(spec_name, classic):
    import multiprocessing as mp
    from hstream_amd.engine import Engine
    G = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"hsgf-{os.getpid()}-{uuid.uuid4().hex[:12]}"
    procs = [ctx.Process(target=_form_worker, args=(r, G, name, spec_name, classic, q)) for r in range(G)]
    for p in procs:
        p.start()
    try:
        outs = [q.get(timeout=100) for _ in range(G)]
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    errs = [o for o in outs if o[1] == "error"]
    assert not errs, errs
    outs.sort(key=lambda o: o[0])
    # one GPU fed the whole stream
    spec = FORM_SPECS[spec_name]
    eng = Engine(device=0, batch_capacity=1 << 14)
    op = eng.op(spec)
    wm, ref = -1, []
    for slices in _form_slices(G):
        key = np.concatenate([s[0] for s in slices])
        ts = np.concatenate([s[1] for s in slices])
        cols = [np.concatenate([s[2][c] for s in slices]) for c in range(2)]
        valid = [np.concatenate([s[3][c] for s in slices]) for c in range(2)]
        wm = op.push(key, ts, cols, valid, watermark=wm)
        ref.append(_form_rows(spec, op.drain()))
    op.close()
    eng.close()
    assert all(o[1] == wm for o in outs)
    for bi in range(len(ref)):
        got = sorted(outs[0][2][bi] + outs[1][2][bi], key=lambda t: (t[3], t[1], t[0], t[2], t[4], repr(t[5])))
        exp = sorted(ref[bi], key=lambda t: (t[3], t[1], t[0], t[2], t[4], repr(t[5])))
        assert len(got) == len(exp), (bi, len(got), len(exp))
        for a, b in zip(got, exp):
            assert a[:5] == b[:5] and _close(a[5], b[5]), (bi, a, b)
