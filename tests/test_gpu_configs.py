"""GPU parity on every BASELINE.json config's workload (C1-C5).

Two kinds of checks:

* reduced sizes the oracle finishes in seconds, compared row for row
  (integers bit-exact, f64 within util.F64_RTOL): C4 at the config's per-key
  arrival density (gap 30 s, mean inter-arrival 72 s per key), C5 with its
  Zipf(1.2) key draw over the 1e8-key universe; C1-C3 are in
  test_gpu_parity.py::test_configs_reduced;
* the configs at full size, through properties that hold at any size and are
  checked on the device: C2 (100M records) conserves COUNT(*) and SUM over the
  state; C4 (500M records, 10M keys) leaves every key's sessions disjoint and
  more than the gap apart, with COUNT(*)/SUM conserved; C5 (100M Zipf records)
  gives the hottest key the SUM/MAX per window of a host reduction of its
  records.

Reference semantics: TimeWindowedStream.hs:72-117 (windows, grace),
SessionWindowedStream.hs:84-118 with the findSessions test of Store.hs:243-272
(a point joins every session with end >= t - gap and start <= t + gap).
"""
import dataclasses

import numpy as np
import pytest

import pyoracle
from hstream_amd import abi, datagen
from util import rows_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import torch
    assert torch.cuda.is_available(), "GPU tests need cuda:0"
    from hstream_amd.engine import Engine
    e = Engine(device=0, batch_capacity=1 << 24)
    yield e
    e.close()


def _drive_cfg(eng, cfg, spec, n, batch, faithful_sessions=True):
    g = eng.op(spec)
    o = pyoracle.OracleOp(spec, faithful_sessions=faithful_sessions)
    f64 = spec.agg_is_f64()
    wg = wo = -1
    for bi, s in enumerate(range(0, n, batch)):
        h = datagen.generate(cfg, n=min(batch, n - s), start=s, total=n)
        cols = h["cols"] if spec.col_types else []
        wg = g.push(h["key_id"], h["ts"], cols, None, watermark=wg)
        wo = o.push(h["key_id"], h["ts"], cols, None, watermark=wo)
        assert wg == wo, f"batch {bi}: watermark {wg} != {wo}"
        if spec.emit_mode != abi.HSG_EMIT_NONE:
            rows_equal(g.drain(), o.drain(), f64, ordered=spec.emit_mode == abi.HSG_EMIT_PER_RECORD,
                       what=f"changelog batch {bi}")
    rows_equal(g.dump_state(), o.dump_state(), f64, what="state dump")
    g.close()
    o.close()


# C4 at its per-key density: 10 records per key over 720 s = 72 s mean
# inter-arrival, as 500M records over 10M keys in one hour
C4_REDUCED = dataclasses.replace(datagen.CONFIGS["C4"], keys=200_000, n=2_000_000, span_ms=720_000)


@pytest.mark.parametrize("mode", [abi.HSG_EMIT_PER_BATCH, abi.HSG_EMIT_PER_RECORD, abi.HSG_EMIT_NONE],
                         ids=["per_batch", "per_record", "none"])
def test_c4_sessions_reduced(eng, mode):
    cfg = C4_REDUCED
    spec = cfg.spec(mode, state_capacity=cfg.n)
    # the fast session store of the oracle (cross-checked against the faithful
    # nested-map store in tests/test_oracle.py) keeps this in seconds
    _drive_cfg(eng, cfg, spec, cfg.n, 1 << 18, faithful_sessions=False)


def test_c2_one_bench_batch_exact(eng):
    """One 2^24-record C2 batch, the bench's batch size (4096 partition tiles:
    the offsets' segment sums take the one-workgroup scan of up to 2^15
    elements), row for row against the oracle."""
    cfg = datagen.CONFIGS["C2"]
    n = 1 << 24
    spec = cfg.spec(abi.HSG_EMIT_PER_BATCH, state_capacity=cfg.keys * 64)
    _drive_cfg(eng, cfg, spec, n, n)


def test_c5_zipf_reduced(eng):
    cfg = datagen.CONFIGS["C5"]
    n = 2_000_000
    spec = cfg.spec(abi.HSG_EMIT_PER_BATCH, state_capacity=n)
    _drive_cfg(eng, cfg, spec, n, 1 << 19)


# ---------------------------------------------------------------------------
# full sizes: properties checked on the device
# ---------------------------------------------------------------------------
def _device_state(op, spec, cap):
    """Dump the op's state into device columns (no host round trip)."""
    import ctypes as C
    import torch
    f64 = spec.agg_is_f64()
    cols = {k: torch.empty(cap, dtype=t, device="cuda") for k, t in
            (("key", torch.int32), ("ws", torch.int64), ("we", torch.int64), ("src", torch.int64))}
    aggs = [torch.empty(cap, dtype=torch.float64 if f else torch.int64, device="cuda") for f in f64]
    ap = (C.c_void_p * len(aggs))(*[a.data_ptr() for a in aggs])
    rows = abi.hsg_rows(capacity=cap, mem=abi.HSG_MEM_DEVICE, n_aggs=len(aggs), key_id=cols["key"].data_ptr(),
                        win_start=cols["ws"].data_ptr(), win_end=cols["we"].data_ptr(),
                        src_index=cols["src"].data_ptr(), aggs=C.cast(ap, C.POINTER(C.c_void_p)))
    got = C.c_uint64(0)
    op._check(op._lib.hsg_dump_state(op._h, C.byref(rows), C.byref(got)), "dump_state")
    n = got.value
    return {k: v[:n] for k, v in cols.items()}, [a[:n] for a in aggs]


def _push_device(op, cfg, n, batch, sums=None):
    """Generate the config on the device batch by batch and push it; returns
    (watermark, host-side reductions of COUNT / SUM of the pushed records)."""
    import torch
    wm = -1
    cnt = 0
    tot = 0
    for s in range(0, n, batch):
        m = min(batch, n - s)
        h = datagen.generate_torch(cfg, m, device="cuda", start=s, total=n)
        torch.cuda.synchronize()
        wm = op.push(h["key_id"], h["ts"], h["cols"] if op.spec.col_types else [], None, watermark=wm)
        cnt += m
        if sums is not None:
            tot += int(h["cols"][0].sum().item())
        del h
    return wm, cnt, tot


def test_c2_full_conservation(eng):
    """C2, 100M records: every record has ts >= 0 and none is late (the ts are
    near-sorted with 2 s jitter, grace 24 h), so COUNT(*) and SUM summed over
    the state equal the record count and the column sum; AVG = SUM / COUNT."""
    import torch
    cfg = datagen.CONFIGS["C2"]
    spec = cfg.spec(abi.HSG_EMIT_NONE, state_capacity=cfg.keys * 64)
    op = eng.op(spec)
    _, cnt, tot = _push_device(op, cfg, cfg.n, cfg.batch, sums=True)
    cols, aggs = _device_state(op, spec, cfg.keys * 64)
    # aggs: COUNT(*), SUM, AVG, MIN, MAX
    assert int(aggs[0].sum().item()) == cnt == cfg.n
    assert int(aggs[1].sum().item()) == tot
    ws = cols["ws"]
    assert bool(((ws % cfg.size_ms) == 0).all()) and bool((cols["we"] - ws == cfg.size_ms).all())
    assert bool((aggs[3] <= aggs[4]).all())
    avg = aggs[1].to(torch.float64) / aggs[0].to(torch.float64)
    assert torch.allclose(aggs[2], avg, rtol=1e-12, atol=0)
    # each (key, window) appears once
    g = cols["key"].to(torch.int64) * (1 << 32) + (ws - datagen.TS0) // cfg.size_ms
    assert int(torch.unique(g).numel()) == int(g.numel())
    op.close()


def test_c3_full_hopping(eng):
    """C3 at full size (1B records, 1M keys, hopping 60 s / 5 s, COUNT(*) +
    SUM): every record is at ts >= 60 s and none is late, so each lands in
    exactly 12 windows (TimeWindowedStream.hs:105-117): COUNT(*) summed over
    the state is 12 x the records, SUM 12 x the column sum, every (key, window)
    has one row, and the table (sized by the groups the batches make, the
    deferred updates' room check) stays at most 2^30 slots for the ~731M
    groups."""
    import torch
    cfg = datagen.CONFIGS["C3"]
    spec = cfg.spec(abi.HSG_EMIT_NONE)
    op = eng.op(spec)
    _, cnt, tot = _push_device(op, cfg, cfg.n, cfg.batch, sums=True)
    st = op.stats()
    live = st["state_rows"]
    cols, aggs = _device_state(op, spec, live)
    assert int(cols["key"].numel()) == live
    assert int(aggs[0].sum().item()) == 12 * cnt and cnt == cfg.n
    assert int(aggs[1].sum().item()) == 12 * tot
    ws = cols["ws"]
    assert bool(((ws % cfg.advance_ms) == 0).all()) and bool((cols["we"] - ws == cfg.size_ms).all())
    g = cols["key"].to(torch.int64) * (1 << 32) + (ws - datagen.TS0 + 3_600_000) // cfg.advance_ms
    del cols, aggs
    g, _ = torch.sort(g)
    assert not bool((g[1:] == g[:-1]).any()), "a (key, window) with two rows"
    op.close()
    print({k: st[k] for k in ("state_rows", "table_slots", "grow_events", "overflow_rebuilds", "replays")})
    # hopping tables run at up to half load: 766M
    # (key, window) rows fit 2^31 slots, sized by the groups, not the updates
    assert st["table_slots"] <= (1 << 31) and 2 * st["state_rows"] <= st["table_slots"], st


def test_c4_full_sessions_disjoint(eng):
    """C4 at full size (500M records, 10M keys, gap 30 s): after every batch
    the sessions of one key are disjoint and more than the gap apart (the
    closure of the per-record merges, Store.hs:243-272), COUNT(*) sums to the
    records pushed and SUM to their column sum."""
    import torch
    cfg = datagen.CONFIGS["C4"]
    spec = cfg.spec(abi.HSG_EMIT_NONE, state_capacity=cfg.n)
    op = eng.op(spec)
    _, cnt, tot = _push_device(op, cfg, cfg.n, cfg.batch, sums=True)
    live = op.stats()["state_rows"]
    cols, aggs = _device_state(op, spec, live)
    assert int(cols["key"].numel()) == live
    assert int(aggs[0].sum().item()) == cnt == cfg.n
    assert int(aggs[1].sum().item()) == tot
    key = cols["key"].to(torch.int64)
    st, en = cols["ws"], cols["we"]
    assert bool((st <= en).all())
    # sort by (key, start); consecutive sessions of one key: next.start - end > gap
    o2 = torch.argsort(st, stable=True)
    o2 = o2[torch.argsort(key[o2], stable=True)]
    k2, s2, e2 = key[o2], st[o2], en[o2]
    same = k2[1:] == k2[:-1]
    gaps = s2[1:] - e2[:-1]
    assert bool((gaps[same] > cfg.gap_ms).all())
    # a session's count is at least 1 and its span covers its count's arrivals
    assert bool((aggs[0] >= 1).all())
    op.close()


def test_c5_full_hot_key(eng):
    """C5 at full size (100M Zipf(1.2) records over the 1e8-key universe): the
    hottest key (rank 0) gets, per window, the SUM and MAX of a host reduction
    of exactly its records; SUM over every group equals the column sum."""
    import torch
    cfg = datagen.CONFIGS["C5"]
    spec = cfg.spec(abi.HSG_EMIT_NONE, state_capacity=1 << 27)
    op = eng.op(spec)
    hot = int(datagen._perm27(np.array([0]))[0])
    wm = -1
    tot = 0
    exp_sum, exp_max = {}, {}
    for s in range(0, cfg.n, cfg.batch):
        m = min(cfg.batch, cfg.n - s)
        h = datagen.generate(cfg, n=m, start=s, total=cfg.n)
        sel = h["key_id"] == hot
        w = (h["ts"][sel] // cfg.size_ms) * cfg.size_ms
        v = h["cols"][0][sel]
        for ws in np.unique(w):
            vv = v[w == ws]
            exp_sum[int(ws)] = exp_sum.get(int(ws), 0) + int(vv.sum())
            exp_max[int(ws)] = max(exp_max.get(int(ws), -(1 << 63)), int(vv.max()))
        tot += int(h["cols"][0].sum())
        wm = op.push(torch.from_numpy(h["key_id"].view(np.int32)).cuda(), torch.from_numpy(h["ts"]).cuda(),
                     [torch.from_numpy(h["cols"][0]).cuda()], None, watermark=wm)
    cols, aggs = _device_state(op, spec, op.stats()["state_rows"])
    assert int(aggs[0].sum().item()) == tot
    sel = cols["key"] == np.int32(np.uint32(hot).view(np.int32))
    got_ws = cols["ws"][sel].cpu().numpy()
    got_sum = aggs[0][sel].cpu().numpy()
    got_max = aggs[1][sel].cpu().numpy()
    assert sorted(got_ws.tolist()) == sorted(exp_sum)
    for ws, sm, mx in zip(got_ws, got_sum, got_max):
        assert int(sm) == exp_sum[int(ws)] and int(mx) == exp_max[int(ws)], ws
    # the hot key really is hot: about 1/zeta(1.2) of the records
    assert sum(exp_sum) > 0 and len(exp_sum) >= 50
    op.close()
