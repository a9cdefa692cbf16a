"""C3 at full size: table growth per batch (diagnostic)."""
import os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import torch
from hstream_amd import abi, datagen
from hstream_amd.engine import Engine

cfg = datagen.CONFIGS["C3"]
eng = Engine(device=0, batch_capacity=cfg.batch)
op = eng.op(cfg.spec(abi.HSG_EMIT_NONE))
wm = -1
for bi, s in enumerate(range(0, cfg.n, cfg.batch)):
    m = min(cfg.batch, cfg.n - s)
    h = datagen.generate_torch(cfg, m, device="cuda", start=s, total=cfg.n)
    torch.cuda.synchronize()
    wm = op.push(h["key_id"], h["ts"], h["cols"], None, watermark=wm)
    st = op.stats()
    print(bi, {k: st[k] for k in ("state_rows", "table_slots", "grow_events", "overflow_rows", "overflow_rebuilds",
                                  "replays", "touched", "pairs")}, flush=True)
op.close()
eng.close()
