"""Debug: the table-room test's batches one by one, stats after each."""
import sys
import numpy as np
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from hstream_amd import abi, datagen
from hstream_amd.columnar import OpSpec
from hstream_amd.engine import Engine

eng = Engine(device=0, batch_capacity=1 << 22)
for cap in (1 << 10, 1 << 20):
    spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[abi.HSG_I64],
                  aggs=datagen.C_AGGS_FULL, state_capacity=cap)
    g = eng.op(spec)
    rng = np.random.default_rng(11)
    t = 10_000_000
    wg = -1
    for bi, (nkeys, span, n) in enumerate([(20_000, 600_000, 300_000), (20_000, 600_000, 300_000),
                                           (5_000, 2_000_000_000, 100_000), (20_000, 600_000, 300_000),
                                           (300_000, 600_000, 400_000), (20_000, 600_000, 300_000)]):
        key = rng.integers(0, nkeys, size=n).astype(np.uint32)
        ts = (t + np.sort(rng.integers(0, span, size=n))).astype(np.int64)
        cols = [rng.integers(-10**9, 10**9, size=n, dtype=np.int64)]
        t += span
        try:
            wg = g.push(key, ts, cols, None, watermark=wg)
        except Exception as e:
            print(f"cap {cap} batch {bi}: {e}", flush=True)
            print({k: v for k, v in g.stats().items()}, flush=True)
            break
        g.drain()
        st = g.stats()
        print(f"cap {cap} batch {bi}: slots {st['table_slots']} grow {st['grow_events']} replays {st['replays']} "
              f"lean {st['lean_batches']} direct {st['direct_batches']} rows {st.get('state_rows')}", flush=True)
    g.close()
eng.close()
