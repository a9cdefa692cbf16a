"""CPU, world_size 2 over gloo: the multi-GPU sharding protocol of
hstream_amd/csrc/exchange.cpp restated with torch.distributed and checked
against one oracle fed the whole batch.

Protocol per global batch (rank r ingests slice r; slices are in rank order):
  all-gather (max ts, min keyed ts, n) -> global watermark, stream-time carry
  of rank r = max(wm_in, max ts of ranks < r), sequence base = sum of n of
  ranks < r, and whether any record may be late (stream time > min ts + grace);
  owner = the top log2(G) bits of key_hash(key) (power-of-two G, the bits the
  local partition skips; hash mod G otherwise);
  fast path (no LAST, no per-record changelog, no sessions, and no record can
  be late): one all-to-all per column of (key, ts, col..., valid...) of the
  keyed records with ts >= 0, aggregated in any order at stream time = carry;
  sequenced path otherwise: the same columnar all-to-all with two more
  columns, each record's global sequence number and (when some record may be
  late) its stream time, the owner partition stable (arrival order kept), of
  the keyed records with ts >= 0 (any ts for sessions and unwindowed ops);
  each rank aggregates its owned records in global order. (A rank count that
  is not a power of two, or HSG_KNOB_X_CLASSIC, takes the packed classic
  exchange: the same records and sequence numbers, one packed all-to-all.)
The per-rank aggregation here is the oracle, so this checks the protocol's
claims (exact stream time and sequence numbers after the exchange, disjoint
key ownership), not the GPU kernels (tests/test_gpu_parity.py does that)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from hstream_amd import abi
from hstream_amd.columnar import OpSpec
from util import ALL_AGG_SETS, gen_small

M64 = (1 << 64) - 1


def mix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xFF51AFD7ED558CCD)
        x = x ^ (x >> np.uint64(33))
        x = x * np.uint64(0xC4CEB9FE1A85EC53)
        x = x ^ (x >> np.uint64(33))
    return x


def fmix32(h):
    """hsg_internal.h fmix32 (murmur3's 32-bit finaliser)"""
    h = np.asarray(h, np.uint32)
    with np.errstate(over="ignore"):
        h = h ^ (h >> np.uint32(16))
        h = h * np.uint32(0x85EBCA6B)
        h = h ^ (h >> np.uint32(13))
        h = h * np.uint32(0xC2B2AE35)
        h = h ^ (h >> np.uint32(16))
    return h


def key_hash(key):
    """hsg_internal.h key_hash: fmix32(key * golden32 + c) in the high word, a
    second mix in the low word"""
    k = np.asarray(key, np.uint32)
    with np.errstate(over="ignore"):
        h = fmix32(k * np.uint32(0x9E3779B1) + np.uint32(0x632BE59B))
        lo = (h * np.uint32(0x27D4EB2F)) ^ k
    return (h.astype(np.uint64) << np.uint64(32)) | lo.astype(np.uint64)


def owner_of(key, G):
    """k_exchange.hip owner_of"""
    lg = G.bit_length() - 1
    if (1 << lg) == G:
        if lg == 0:
            return np.zeros(len(key), np.int64)
        return (key_hash(key) >> np.uint64(64 - lg)).astype(np.int64)
    return (mix64(np.asarray(key, np.uint64) ^ np.uint64(0x5BD1E9955BD1E995)) % np.uint64(G)).astype(np.int64)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


SPECS = {
    "hopping": OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_RECORD, size_ms=10_000, advance_ms=3_000,
                      col_types=[abi.HSG_I64, abi.HSG_F64], aggs=ALL_AGG_SETS["mixed"]),
    "tumbling_batch": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000,
                             col_types=[abi.HSG_I64, abi.HSG_F64], aggs=ALL_AGG_SETS["mixed"]),
    "session": OpSpec(abi.HSG_SESSION, abi.HSG_EMIT_PER_RECORD, gap_ms=2_000, col_types=[abi.HSG_I64, abi.HSG_F64],
                      aggs=ALL_AGG_SETS["mixed"]),
    # no LAST: the fast exchange when no record can be late
    "tumbling_fast": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000,
                            col_types=[abi.HSG_I64, abi.HSG_F64],
                            aggs=[a for a in ALL_AGG_SETS["mixed"] if a[0] != abi.HSG_LAST]),
    "hopping_fast": OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_NONE, size_ms=9_000, advance_ms=3_000,
                           col_types=[abi.HSG_I64, abi.HSG_F64],
                           aggs=[a for a in ALL_AGG_SETS["mixed"] if a[0] != abi.HSG_LAST]),
    # no LAST but a short grace: batches whose records may be late take the sequenced exchange
    "tumbling_fast_grace": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, grace_ms=5_000,
                                  col_types=[abi.HSG_I64, abi.HSG_F64],
                                  aggs=[a for a in ALL_AGG_SETS["mixed"] if a[0] != abi.HSG_LAST]),
}
# the exchange each spec takes on these batches (very late records have ts < 0: never windowed)
PATHS = {"hopping": "sequenced", "tumbling_batch": "sequenced", "session": "sequenced", "tumbling_fast": "fast",
         "hopping_fast": "fast", "tumbling_fast_grace": "sequenced"}


def fast_eligible(spec):
    """exchange.cpp push_sharded: no LAST, per-record changelog or sessions"""
    return (spec.emit_mode != abi.HSG_EMIT_PER_RECORD and spec.window_kind != abi.HSG_SESSION
            and all(k != abi.HSG_LAST for k, _ in spec.aggs))


def _batches(G, late):
    out = []
    for bi in range(3):
        slices = []
        for r in range(G):
            slices.append(gen_small(500 + 10 * bi + r, 1500, 23, col_types=(abi.HSG_I64, abi.HSG_F64),
                                    span=30_000, base=2_000_000 + bi * 30_000 + r * 7_000, very_late=late))
        out.append(slices)
    return out


def _worker(rank, G, port, spec_name, late, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=G)
    import pyoracle
    spec = SPECS[spec_name]
    op = pyoracle.OracleOp(spec)
    wm = -1
    rec_base = 0
    results = []
    paths = []
    for slices in _batches(G, late):
        key, ts, cols, valid = slices[rank]
        keyed = key != abi.HSG_KEY_NONE
        mn = int(ts[keyed & (ts >= 0)].min()) if (keyed & (ts >= 0)).any() else np.iinfo(np.int64).max
        facts = torch.tensor([int(ts.max()) if len(ts) else np.iinfo(np.int64).min, mn, len(ts)], dtype=torch.int64)
        allf = [torch.zeros(3, dtype=torch.int64) for _ in range(G)]
        dist.all_gather(allf, facts)
        allf = [f.tolist() for f in allf]
        carry = max([wm] + [f[0] for q_, f in enumerate(allf) if q_ < rank and f[2] > 0])
        wm_global = max([wm] + [f[0] for f in allf if f[2] > 0])
        min_ts = min(f[1] for f in allf if f[2] > 0)
        seq_base = rec_base + sum(f[2] for q_, f in enumerate(allf) if q_ < rank)
        total = sum(f[2] for f in allf)
        time_win = spec.window_kind in (abi.HSG_TUMBLING, abi.HSG_HOPPING)
        may_be_late = time_win and wm_global > min_ts + spec.grace_ms
        if fast_eligible(spec) and not may_be_late:
            # fast path: keyed records with ts >= 0 (any ts for unwindowed), one all-to-all per column
            sel = keyed & ((ts >= 0) | (spec.window_kind == abi.HSG_UNWINDOWED))
            own = np.where(sel, owner_of(key, G), G)
            order = np.argsort(own, kind="stable")
            order = order[own[order] < G]
            counts = np.bincount(own[own < G], minlength=G)
            rcnt = torch.zeros(G, dtype=torch.int64)
            dist.all_to_all_single(rcnt, torch.from_numpy(counts.astype(np.int64)))
            cols_in = [key.astype(np.int64), ts, cols[0], cols[1].view(np.int64), valid[0].astype(np.int64),
                       valid[1].astype(np.int64)]
            cols_out = []
            for col in cols_in:
                send = torch.from_numpy(np.ascontiguousarray(col[order]))
                recv = torch.zeros(int(rcnt.sum()), dtype=torch.int64)
                dist.all_to_all_single(recv, send, [int(c) for c in rcnt], [int(c) for c in counts])
                cols_out.append(recv.numpy())
            op.push_ex(cols_out[0].astype(np.uint32), cols_out[1].copy(),
                       [cols_out[2].copy(), cols_out[3].copy().view(np.float64)],
                       [cols_out[4].astype(np.uint8), cols_out[5].astype(np.uint8)], watermark=carry)
            paths.append("fast")
        else:
            rec_wm = np.maximum.accumulate(np.concatenate([[carry], ts]))[1:]
            seq = seq_base + np.arange(len(ts), dtype=np.int64)
            all_ts = spec.window_kind in (abi.HSG_SESSION, abi.HSG_UNWINDOWED)
            own = np.where(keyed & ((ts >= 0) | all_ts), owner_of(key, G), G)
            # stable partition by owner, drop HSG_KEY_NONE
            order = np.argsort(own, kind="stable")
            order = order[own[order] < G]
            counts = np.bincount(own[own < G], minlength=G)
            rows = np.stack([key.astype(np.int64), ts, cols[0], cols[1].view(np.int64), valid[0].astype(np.int64),
                             valid[1].astype(np.int64), seq, rec_wm], axis=1)[order]
            send = torch.from_numpy(np.ascontiguousarray(rows)).reshape(-1)
            cnt_t = torch.from_numpy(counts.astype(np.int64))
            rcnt = torch.zeros(G, dtype=torch.int64)
            dist.all_to_all_single(rcnt, cnt_t)
            recv = torch.zeros(int(rcnt.sum()) * 8, dtype=torch.int64)
            dist.all_to_all_single(recv, send, [int(c) * 8 for c in rcnt], [int(c) * 8 for c in counts])
            got = recv.reshape(-1, 8).numpy()
            r_key = got[:, 0].astype(np.uint32)
            r_cols = [got[:, 2].copy(), got[:, 3].copy().view(np.float64)]
            r_valid = [got[:, 4].astype(np.uint8), got[:, 5].astype(np.uint8)]
            op.push_ex(r_key, got[:, 1].copy(), r_cols, r_valid, watermark=carry,
                       rec_wm=got[:, 7].copy() if may_be_late else None, seq=got[:, 6].copy())
            paths.append("sequenced")
        wm = wm_global
        rec_base += total
        rows_out = op.drain() if spec.emit_mode != abi.HSG_EMIT_NONE else None
        if rows_out is not None and spec.emit_mode == abi.HSG_EMIT_PER_BATCH:
            rows_out.src_index[:] = -1  # per-batch rows carry no producing record
        results.append(None if rows_out is None else rows_out.tuples_with_src() if hasattr(rows_out, "tuples_with_src")
                       else [(int(rows_out.key_id[i]), int(rows_out.win_start[i]), int(rows_out.win_end[i]),
                              int(rows_out.src_index[i]), tuple(a[i].item() for a in rows_out.aggs))
                             for i in range(len(rows_out))])
    state = op.dump_state().tuples()
    q.put((rank, wm, results, state, paths))
    dist.destroy_process_group()


def _single(spec_name, G, late):
    import pyoracle
    spec = SPECS[spec_name]
    op = pyoracle.OracleOp(spec)
    wm = -1
    results = []
    for slices in _batches(G, late):
        key = np.concatenate([s[0] for s in slices])
        ts = np.concatenate([s[1] for s in slices])
        cols = [np.concatenate([s[2][c] for s in slices]) for c in range(2)]
        valid = [np.concatenate([s[3][c] for s in slices]) for c in range(2)]
        wm = op.push(key, ts, cols, valid, watermark=wm)
        if spec.emit_mode == abi.HSG_EMIT_NONE:
            results.append(None)
            continue
        r = op.drain()
        if spec.emit_mode == abi.HSG_EMIT_PER_BATCH:
            r.src_index[:] = -1
        results.append([(int(r.key_id[i]), int(r.win_start[i]), int(r.win_end[i]), int(r.src_index[i]),
                         tuple(a[i].item() for a in r.aggs)) for i in range(len(r))])
    return wm, results, op.dump_state().tuples()


def _close(a, b):
    for x, y in zip(a, b):
        if isinstance(x, float) or isinstance(y, float):
            if not (np.isnan(x) and np.isnan(y)) and abs(x - y) > 1e-9 * max(1.0, abs(x), abs(y)):
                return False
        elif x != y:
            return False
    return True


@pytest.mark.parametrize("late", [False, True], ids=["no_late", "late"])
@pytest.mark.parametrize("spec_name", list(SPECS))
def test_two_rank_protocol_equals_single_stream(spec_name, late):
    G = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, G, port, spec_name, late, q)) for r in range(G)]
    for p in procs:
        p.start()
    outs = [q.get(timeout=240) for _ in range(G)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs.sort()
    wm1, res1, st1 = _single(spec_name, G, late)
    assert all(o[1] == wm1 for o in outs)
    # which exchange ran: the fast one when eligible and no record can be late
    for o in outs:
        assert set(o[4]) == {PATHS[spec_name]}, o[4]
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
        rows = sorted(outs[0][2][bi] + outs[1][2][bi], key=lambda t: (t[3], t[1], t[0], t[2]))
        ref = sorted(res1[bi], key=lambda t: (t[3], t[1], t[0], t[2]))
        assert len(rows) == len(ref)
        for a, b in zip(rows, ref):
            assert a[:4] == b[:4] and _close(a[4], b[4]), (a, b)
