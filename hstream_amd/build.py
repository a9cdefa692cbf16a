"""Build libhstream_gpu.so in-tree (hipcc, --offload-arch=gfx950)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")


def build(jobs=8, verbose=False):
    cmd = ["make", "-C", CSRC, f"-j{jobs}"]
    if not verbose:
        cmd.insert(1, "-s")
    subprocess.check_call(cmd)
    return os.path.join(HERE, "libhstream_gpu.so")


if __name__ == "__main__":
    print(build(verbose=True))
