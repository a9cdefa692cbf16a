"""Phase clocks of one config's batches (diagnostic): loads a PHASES=1 build
(make -C hstream_amd/csrc PHASES=1 OUT=../phases_lib/libhstream_gpu.so
BUILD=../../build/hsg_phases) and pushes a few device batches; the library
prints [hsg phases] lines to stderr when HSG_PHASES is set.
  HSG_PHASES=1 python tools/dbg/phases.py C4 [batches]"""
import os, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch
from hstream_amd import abi, datagen, engine
engine.load_library(os.path.join(ROOT, "hstream_amd", "phases_lib", "libhstream_gpu.so"))
from hstream_amd.engine import Engine

cfg = datagen.CONFIGS[sys.argv[1]]
nb = int(sys.argv[2]) if len(sys.argv) > 2 else 12
eng = Engine(device=0, batch_capacity=cfg.batch)
emit = {"none": abi.HSG_EMIT_NONE, "per_record": abi.HSG_EMIT_PER_RECORD}[sys.argv[3] if len(sys.argv) > 3 else "none"]
op = eng.op(cfg.spec(emit, out_capacity=cfg.batch * 16 if emit == abi.HSG_EMIT_PER_RECORD else 0))
wm = -1
for bi in range(nb):
    s = bi * cfg.batch
    h = datagen.generate_torch(cfg, cfg.batch, device="cuda", start=s, total=cfg.n)
    torch.cuda.synchronize()
    print(f"batch {bi}", file=sys.stderr, flush=True)
    wm = op.push(h["key_id"], h["ts"], h["cols"], None, watermark=wm)
    if emit != abi.HSG_EMIT_NONE:
        op.drain()
op.close()
eng.close()
