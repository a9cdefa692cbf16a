"""ctypes binding of libhstream_gpu (the product path).

Loads the in-tree ``hstream_amd/libhstream_gpu.so``; there is no fallback of
any kind: if the library is missing or the GPU is absent, constructing an
Engine raises.
"""
import ctypes as C
import os

from . import abi
from .columnar import OpHandle, OpSpec, declare_op_functions

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libhstream_gpu.so")
# diagnostics only: HSG_LIB_PATH names another build of the same library
# (e.g. the PHASES=1 phase-clock build, tools/phases.sh)
LIB_PATH = os.environ.get("HSG_LIB_PATH", LIB_PATH)
_lib = None


def load_library(path=LIB_PATH):
    """Load libhstream_gpu.so and declare every exported signature."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(
            f"libhstream_gpu.so not found at {path}: run __graft_entry__.build() "
            "(the GPU path has no fallback)")
    L = C.CDLL(path)
    vp = C.c_void_p
    P = C.POINTER
    L.hsg_comm_unique_id.argtypes = [P(C.c_uint8), C.c_size_t]
    L.hsg_comm_unique_id.restype = C.c_int
    L.hsg_engine_create.argtypes = [P(abi.hsg_engine_config), P(vp)]
    L.hsg_engine_create.restype = C.c_int
    L.hsg_engine_destroy.argtypes = [vp]
    L.hsg_engine_destroy.restype = None
    L.hsg_engine_last_error.argtypes = [vp]
    L.hsg_engine_last_error.restype = C.c_char_p
    L.hsg_op_create.argtypes = [vp, P(abi.hsg_op_config), P(vp)]
    L.hsg_op_create.restype = C.c_int
    L.hsg_op_stats.argtypes = [vp, P(abi.hsg_stats)]
    L.hsg_op_stats.restype = C.c_int
    L.hsg_op_set_changelog.argtypes = [vp, P(abi.hsg_rows)]
    L.hsg_op_set_changelog.restype = C.c_int
    L.hsg_push_batch_async.argtypes = [vp, P(abi.hsg_batch), P(C.c_int64), abi.HSG_DONE_FN, vp]
    L.hsg_push_batch_async.restype = C.c_int
    L.hsg_op_wait.argtypes = [vp]
    L.hsg_op_wait.restype = C.c_int
    L.hsg_testing_set_knob.argtypes = [C.c_int32, C.c_int64]
    L.hsg_testing_set_knob.restype = C.c_int
    declare_op_functions(L, "hsg")
    _lib = L
    return L


class testing_knob:
    """Context manager over hsg_testing_set_knob (tests only): the knob holds
    for ops created inside the block, then returns to its default."""

    DEFAULTS = {abi.HSG_KNOB_XPART_LOG2: -1, abi.HSG_KNOB_SESS_ARENA_MIN: 0, abi.HSG_KNOB_X_CLASSIC: 0}

    def __init__(self, knob, value):
        self.knob, self.value = knob, value

    def __enter__(self):
        rc = load_library().hsg_testing_set_knob(self.knob, self.value)
        if rc != abi.HSG_OK:
            raise abi.HStreamGpuError(rc, "hsg_testing_set_knob")
        return self

    def __exit__(self, *exc):
        load_library().hsg_testing_set_knob(self.knob, self.DEFAULTS[self.knob])
        return False


def comm_unique_id() -> bytes:
    L = load_library()
    buf = (C.c_uint8 * abi.HSG_COMM_ID_BYTES)()
    rc = L.hsg_comm_unique_id(buf, abi.HSG_COMM_ID_BYTES)
    if rc != abi.HSG_OK:
        raise abi.HStreamGpuError(rc, "hsg_comm_unique_id")
    return bytes(buf)


class Engine:
    """One per process and GPU (hsg_engine_create)."""

    def __init__(self, device=0, rank=0, nranks=1, comm_id=None, batch_capacity=1 << 24,
                 transport=abi.HSG_TRANSPORT_RCCL):
        """comm_id: RCCL id bytes (comm_unique_id() on rank 0) or, with
        transport=HSG_TRANSPORT_HOST, a segment name (str / bytes) shared by
        the ranks of one host."""
        L = load_library()
        self._lib = L
        self._id_buf = None
        cfg = abi.hsg_engine_config(device=device, rank=rank, nranks=nranks, transport=transport,
                                    comm_id=None, batch_capacity=batch_capacity)
        if isinstance(comm_id, str):
            comm_id = comm_id.encode()
        if comm_id is not None and transport == abi.HSG_TRANSPORT_HOST:
            comm_id = comm_id[: abi.HSG_COMM_ID_BYTES - 1].ljust(abi.HSG_COMM_ID_BYTES, b"\0")
        if comm_id is not None:
            self._id_buf = (C.c_uint8 * abi.HSG_COMM_ID_BYTES)(*comm_id[: abi.HSG_COMM_ID_BYTES])
            cfg.comm_id = C.cast(self._id_buf, P_u8)
        h = C.c_void_p()
        rc = L.hsg_engine_create(C.byref(cfg), C.byref(h))
        if rc != abi.HSG_OK:
            raise abi.HStreamGpuError(rc, "hsg_engine_create")
        self._h = h
        self.device, self.rank, self.nranks, self.batch_capacity = device, rank, nranks, batch_capacity

    def op(self, spec: OpSpec) -> "GpuOp":
        return GpuOp(self, spec)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.hsg_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


P_u8 = C.POINTER(C.c_uint8)


class GpuOp(OpHandle):
    """One windowed GROUP BY operator on the GPU (hsg_op_create)."""

    def __init__(self, engine: Engine, spec: OpSpec):
        cfg, keep = spec.to_config()
        h = C.c_void_p()
        rc = engine._lib.hsg_op_create(engine._h, C.byref(cfg), C.byref(h))
        if rc != abi.HSG_OK:
            msg = engine._lib.hsg_engine_last_error(engine._h)
            raise abi.HStreamGpuError(rc, f"hsg_op_create: {msg.decode() if msg else ''}")
        self.engine = engine  # keep the engine alive while the op lives
        super().__init__(engine._lib, "hsg", h, spec)

    def set_changelog(self, rows):
        """Register caller-owned device columns (an abi.hsg_rows with mem =
        HSG_MEM_DEVICE) as the changelog: pushes write rows there directly and
        drain_count() reports how many (hsg_op_set_changelog). None restores
        the op's own buffer."""
        self._check(self._lib.hsg_op_set_changelog(self._h, C.byref(rows) if rows is not None else None),
                    "op_set_changelog")
        self._sink = rows

    def drain_count(self) -> int:
        """hsg_drain with a registered changelog: the rows are already in place."""
        got = C.c_uint64(0)
        self._check(self._lib.hsg_drain(self._h, None, C.byref(got)), "drain")
        return got.value

    def push_async(self, key_id, ts, cols=(), valid=None, watermark=None, done=None, mem=None, **enc):
        """hsg_push_batch_async: queue the batch and return at once. `watermark`
        is a ctypes.c_int64 shared by consecutive pushes (read when the batch
        starts, written before `done(rc)` runs on the op's completion thread).
        The arrays are kept alive until the completion has run."""
        from .columnar import make_batch
        b, keep = make_batch(key_id, ts, cols, valid, mem, **enc)
        wm = watermark if watermark is not None else C.c_int64(-1)
        entry = {}

        def _cb(_ctx, rc):
            try:
                if done is not None:
                    done(rc)
            finally:
                self._inflight.pop(id(entry), None)

        cb = abi.HSG_DONE_FN(_cb)
        entry.update(keep=keep, b=b, cb=cb, wm=wm)
        if not hasattr(self, "_inflight"):
            self._inflight = {}
        self._inflight[id(entry)] = entry
        rc = self._lib.hsg_push_batch_async(self._h, C.byref(b), C.byref(wm), cb, None)
        if rc != abi.HSG_OK:
            self._inflight.pop(id(entry), None)
        self._check(rc, "push_batch_async")
        return wm

    def wait(self):
        """hsg_op_wait: block until the queued pushes are done; raises the first failure."""
        self._check(self._lib.hsg_op_wait(self._h), "op_wait")

    def stats(self) -> dict:
        s = abi.hsg_stats()
        self._check(self._lib.hsg_op_stats(self._h, C.byref(s)), "op_stats")
        return s.as_dict()
