"""GPU: hsg_op_reset after the state has been written by every claim path
(lean one-window apply, hopping pane apply, per-record changelog, a table
grown mid-run). The reset rewrites only the blocks the claims marked
(k_tw_reset_dirty), so after it the op must behave exactly like a fresh one:
its changelog and dump compared with a fresh CPU oracle fed only the batches
after the reset (TimeWindowedStream.hs:86-103 per (key, window) group)."""
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


def _batch(rng, n, nkeys, t0, span):
    key = rng.integers(0, nkeys, size=n).astype(np.uint32)
    ts = (t0 + np.sort(rng.integers(0, span, size=n))).astype(np.int64)
    return key, ts, [rng.integers(-10**6, 10**6, size=n, dtype=np.int64)]


SPECS = {
    "tumbling_lean": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[abi.HSG_I64],
                            aggs=datagen.C_AGGS_FULL, state_capacity=1 << 18),
    "hopping_panes": OpSpec(abi.HSG_HOPPING, abi.HSG_EMIT_PER_BATCH, size_ms=60_000, advance_ms=5_000,
                            col_types=[abi.HSG_I64], aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_SUM, 0)],
                            state_capacity=1 << 20),
    "per_record": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_RECORD, size_ms=10_000, col_types=[abi.HSG_I64],
                         aggs=[(abi.HSG_SUM, 0), (abi.HSG_MAX, 0)], state_capacity=1 << 16),
    # a table of 2^12 slots grows (rebuild + reinsert) within the first run
    "grown": OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=1_000, col_types=[abi.HSG_I64],
                    aggs=[(abi.HSG_COUNT_ALL, 0), (abi.HSG_MIN, 0)], state_capacity=1 << 11),
}


@pytest.mark.parametrize("name", list(SPECS))
def test_reset_after_every_claim_path(eng, name):
    spec = SPECS[name]
    f64 = spec.agg_is_f64()
    n = 20_000 if spec.emit_mode == abi.HSG_EMIT_PER_RECORD else 150_000
    rng = np.random.default_rng(17)
    g = eng.op(spec)
    for rnd in range(3):
        o = pyoracle.OracleOp(spec)
        wg = wo = -1
        t = 10_000_000 * (rnd + 1)
        for bi in range(3):
            key, ts, cols = _batch(rng, n, 3_000 * (rnd + 1), t, 400_000)
            t += 400_000
            wg = g.push(key, ts, cols, None, watermark=wg)
            wo = o.push(key, ts, cols, None, watermark=wo)
            assert wg == wo, f"round {rnd} batch {bi}"
            rows_equal(g.drain(), o.drain(), f64, what=f"round {rnd} changelog {bi}")
        rows_equal(g.dump_state(), o.dump_state(), f64, what=f"round {rnd} dump")
        o.close()
        g.reset()
        assert len(g.dump_state()) == 0
    if name == "grown":
        assert g.stats()["grow_events"] >= 1
    g.close()
