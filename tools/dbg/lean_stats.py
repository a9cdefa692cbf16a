import sys, os, numpy as np
sys.path.insert(0, os.getcwd())
sys.path.insert(0, "tests"); sys.path.insert(0, "oracle")
from test_gpu_lean import _batches
from hstream_amd import abi, datagen
from hstream_amd.columnar import OpSpec
from hstream_amd.engine import Engine
e = Engine(device=0, batch_capacity=1 << 22)
spec = OpSpec(abi.HSG_TUMBLING, abi.HSG_EMIT_PER_BATCH, size_ms=10_000, col_types=[abi.HSG_I64], aggs=datagen.C_AGGS_FULL, state_capacity=1 << 20)
g = e.op(spec); wg = -1
for bi, (k, t, c) in enumerate(_batches(5)):
    wg = g.push(k, t, c, None, watermark=wg); g.drain()
    st = g.stats(); print(bi, {x: st[x] for x in ("lean_batches", "direct_batches", "replays", "touched", "table_slots")}, flush=True)
