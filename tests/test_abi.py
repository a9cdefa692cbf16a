"""CPU: the C-ABI library builds for gfx950, loads, and exports exactly what
include/hstream_gpu.h declares; the ctypes mirror matches the C layout."""
import ctypes as C
import os
import re
import subprocess
import tempfile

import pytest

from hstream_amd import abi, engine

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("hstream_gpu.h", "hstream_ingest.h", "hstream_sink.h", "hstream_join.h")]


def _header_functions():
    src = "".join(open(h).read() for h in HEADERS)
    return sorted(set(re.findall(r"^\s*(?:int|void|uint64_t|const char \*)\s*\*?\s*(hsg_\w+)\s*\(", src, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(engine.LIB_PATH):
        from hstream_amd import build
        build.build()
    return engine.load_library()


def test_header_lists_every_abi_function():
    assert _header_functions() == sorted(abi.EXPORTED_SYMBOLS + abi.INGEST_SYMBOLS + abi.SINK_SYMBOLS + abi.JOIN_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.check_output(["nm", "-D", "--defined-only", engine.LIB_PATH]).decode()
    exported = set(re.findall(r" T (hsg_\w+)", out))
    missing = [s for s in _header_functions() if s not in exported]
    assert not missing, missing
    for s in _header_functions():
        assert getattr(lib, s) is not None


def test_library_has_gfx950_code_object(lib):
    blob = open(engine.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_ctypes_layout_matches_c():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "layout")
        subprocess.check_call(["gcc", "-std=c99", "-o", exe, os.path.join(ROOT, "tests", "abi_layout.c")])
        lines = subprocess.check_output([exe]).decode().split("\n")
    want = {}
    for ln in lines:
        if ln.strip():
            k, v = ln.split()
            want[k] = int(v)
    types = {"hsg_engine_config": abi.hsg_engine_config, "hsg_agg": abi.hsg_agg, "hsg_op_config": abi.hsg_op_config,
             "hsg_batch": abi.hsg_batch, "hsg_rows": abi.hsg_rows, "hsg_stats": abi.hsg_stats,
             "hsg_decoder_config": abi.hsg_decoder_config, "hsg_decode_buffers": abi.hsg_decode_buffers,
             "hsg_sink_config": abi.hsg_sink_config, "hsg_sink_records": abi.hsg_sink_records,
             "hsg_sink_spellings": abi.hsg_sink_spellings,
             "hsg_join_config": abi.hsg_join_config, "hsg_join_batch": abi.hsg_join_batch,
             "hsg_join_rows": abi.hsg_join_rows}
    for k, v in want.items():
        if "." in k:
            t, m = k.split(".")
            assert getattr(types[t], m).offset == v, k
        else:
            assert C.sizeof(types[k]) == v, k


def test_engine_create_fails_loudly_without_gpu(lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(abi.HStreamGpuError):
        engine.Engine(device=0)
