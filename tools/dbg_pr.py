"""Debug: per-record changelog on small inputs, GPU vs oracle, printed."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import numpy as np
import pyoracle
from hstream_amd import abi
from hstream_amd.columnar import OpSpec
from hstream_amd.engine import Engine

eng = Engine(device=0, batch_capacity=1 << 16)
def run(name, key, ts, kind=abi.HSG_TUMBLING, **kw):
    spec = OpSpec(kind, abi.HSG_EMIT_PER_RECORD, aggs=[(abi.HSG_COUNT_ALL, 0)], **kw)
    g, o = eng.op(spec), pyoracle.OracleOp(spec)
    g.push(key, ts, [], None); o.push(key, ts, [], None)
    a, b = g.drain(), o.drain()
    ok = len(a) == len(b) and np.array_equal(a.aggs[0], b.aggs[0]) and np.array_equal(a.key_id, b.key_id)
    print(name, "OK" if ok else "FAIL", "n", len(a), len(b))
    if not ok:
        print(" gpu key", a.key_id[:24].tolist()); print(" gpu cnt", a.aggs[0][:24].tolist())
        print(" ref key", b.key_id[:24].tolist()); print(" ref cnt", b.aggs[0][:24].tolist())
    g.close(); o.close()

n = 20
key = (np.arange(n) % 2).astype(np.uint32)
ts = (1_000_000 + np.arange(n)).astype(np.int64)
run("tiny_opt", key, ts, size_ms=10_000)
ts2 = ts.copy(); ts2[5] -= 100_000_000
run("tiny_late", key, ts2, size_ms=10_000)
rng = np.random.default_rng(1)
key3 = rng.integers(0, 37, 5000).astype(np.uint32)
ts3 = (10_000_000 + np.arange(5000) * 20 + rng.integers(0, 3000, 5000)).astype(np.int64)
run("mid_opt", key3, ts3, size_ms=10_000)
ts4 = ts3.copy(); ts4[::50] -= 100_000_000
run("mid_late", key3, ts4, size_ms=10_000)
key5 = rng.integers(0, 3, 60000).astype(np.uint32)
ts5 = (10_000_000 + np.arange(60000)).astype(np.int64)
run("span_chunks", key5, ts5, size_ms=10_000)
