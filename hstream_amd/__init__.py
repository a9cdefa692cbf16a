"""hstream_amd — MI355X-native engine for HStreamDB's windowed GROUP BY path.

The product is the C-ABI library ``libhstream_gpu.so`` (HIP kernels for gfx950,
sources in ``csrc/``, ABI in ``include/hstream_gpu.h``). This package holds its
Python binding and a mirror of the reference's DSL / SQL dispatch surface used
by the tests and the benchmark.
"""
from . import abi  # noqa: F401
from .columnar import OpSpec, Rows  # noqa: F401
