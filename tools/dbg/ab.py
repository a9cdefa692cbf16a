"""bench.py on a variant build of the library (A/B of a build-time constant):
  make -C hstream_amd/csrc OUT=../variants/NAME/libhstream_gpu.so BUILD=../../build/NAME HIPFLAGS+=-D...
  python tools/dbg/ab.py hstream_amd/variants/NAME/libhstream_gpu.so [bench args...]"""
import os, runpy, sys
ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # (HIP runtime first, as bench.py does, then the library)
from hstream_amd import engine
engine.load_library(os.path.abspath(sys.argv[1]))
sys.argv = ["bench.py"] + sys.argv[2:]
runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")
