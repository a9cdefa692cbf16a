import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libhstream_gpu on cuda:0)")
    config.addinivalue_line("markers", "slow: larger sizes")


def pytest_sessionstart(session):
    """GPU runs: torch's HIP runtime first. torch carries its own ROCm
    libraries; when libhstream_gpu (linked against /opt/rocm) initialises the
    device first -- a GPU test file that needs no torch running before one
    that does -- torch.cuda.is_available() can then come back False."""
    mexpr = (getattr(session.config.option, "markexpr", "") or "").replace(" ", "")
    if mexpr == "gpu":
        import torch
        torch.cuda.is_available()
