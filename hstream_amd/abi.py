"""ctypes mirror of include/hstream_gpu.h (structs, enums, status codes).

Kept in one place so the product binding (``hstream_amd.engine``) and the test
oracle binding (``oracle/pyoracle.py``) describe the exact same ABI.
"""
import ctypes as C

HSG_OK = 0
HSG_E_INVALID = -1
HSG_E_OOM = -2
HSG_E_CAPACITY = -3
HSG_E_DEVICE = -4
HSG_E_COMM = -5
HSG_E_RANGE = -6

STATUS_NAMES = {
    HSG_OK: "HSG_OK",
    HSG_E_INVALID: "HSG_E_INVALID",
    HSG_E_OOM: "HSG_E_OOM",
    HSG_E_CAPACITY: "HSG_E_CAPACITY",
    HSG_E_DEVICE: "HSG_E_DEVICE",
    HSG_E_COMM: "HSG_E_COMM",
    HSG_E_RANGE: "HSG_E_RANGE",
}

HSG_KEY_NONE = 0xFFFFFFFF
HSG_TRANSPORT_RCCL = 0
HSG_TRANSPORT_HOST = 1
HSG_COMM_ID_BYTES = 128
HSG_DEFAULT_GRACE_MS = 86400000

# hsg_window_kind
HSG_TUMBLING = 0
HSG_HOPPING = 1
HSG_SESSION = 2
HSG_UNWINDOWED = 3

# hsg_emit_mode
HSG_EMIT_PER_RECORD = 0
HSG_EMIT_PER_BATCH = 1
HSG_EMIT_NONE = 2

# hsg_col_type
HSG_I64 = 0
HSG_F64 = 1

# hsg_agg_kind
HSG_COUNT_ALL = 0
HSG_COUNT = 1
HSG_SUM = 2
HSG_MIN = 3
HSG_MAX = 4
HSG_AVG = 5
HSG_LAST = 6

# hsg_mem
HSG_MEM_HOST = 0
HSG_MEM_DEVICE = 1

# narrow transport encodings (hsg_batch ts_enc / col_enc)
HSG_ENC_FULL = 0
HSG_ENC_TS32 = 1
HSG_ENC_I32 = 2
HSG_ENC_DEC32 = 3
HSG_ENC_K16 = 4
HSG_ENC_TS16 = 5
HSG_TS16_FRAME = 4096
# hsg_batch_narrow / hsg_decode_json_batch: encodings the consumer accepts (hstream_ingest.h)
HSG_NARROW_K16 = 1
HSG_NARROW_TS16 = 2
HSG_NARROW_TS32 = 4
HSG_NARROW_I32 = 8
HSG_NARROW_DEC32 = 16
HSG_NARROW_ALL = 31

# hsg_op_config.flags
HSG_OPF_LITERAL_FORMS = 1


class hsg_engine_config(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("rank", C.c_int32),
        ("nranks", C.c_int32),
        ("transport", C.c_int32),
        ("comm_id", C.POINTER(C.c_uint8)),
        ("batch_capacity", C.c_uint64),
    ]


class hsg_agg(C.Structure):
    _fields_ = [("kind", C.c_int32), ("column", C.c_int32)]


class hsg_op_config(C.Structure):
    _fields_ = [
        ("window_kind", C.c_int32),
        ("emit_mode", C.c_int32),
        ("size_ms", C.c_int64),
        ("advance_ms", C.c_int64),
        ("gap_ms", C.c_int64),
        ("grace_ms", C.c_int64),
        ("n_cols", C.c_int32),
        ("n_aggs", C.c_int32),
        ("col_types", C.POINTER(C.c_int32)),
        ("aggs", C.POINTER(hsg_agg)),
        ("state_capacity", C.c_uint64),
        ("out_capacity", C.c_uint64),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint32),
    ]


class hsg_batch(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("mem", C.c_int32),
        ("n_cols", C.c_int32),
        ("key_id", C.c_void_p),
        ("ts", C.c_void_p),
        ("cols", C.POINTER(C.c_void_p)),
        ("valid", C.POINTER(C.c_void_p)),
        ("ready_event", C.c_void_p),
        ("ts_enc", C.c_int32),
        ("key_enc", C.c_int32),
        ("ts_base", C.c_int64),
        ("col_enc", C.c_uint8 * 8),
        ("col_scale", C.c_uint8 * 8),
        ("ts_frames", C.c_void_p),
    ]


class hsg_decode_buffers(C.Structure):
    _fields_ = [
        ("capacity", C.c_uint64),
        ("key_id", C.c_void_p),
        ("ts", C.c_void_p),
        ("ts_frames", C.c_void_p),
        ("cols", C.POINTER(C.c_void_p)),
        ("valid", C.POINTER(C.c_void_p)),
        ("allow", C.c_uint32),
        ("reserved", C.c_uint32),
        ("col_ptrs", C.c_void_p * 8),
        ("valid_ptrs", C.c_void_p * 8),
    ]


class hsg_rows(C.Structure):
    _fields_ = [
        ("capacity", C.c_uint64),
        ("mem", C.c_int32),
        ("n_aggs", C.c_int32),
        ("key_id", C.c_void_p),
        ("win_start", C.c_void_p),
        ("win_end", C.c_void_p),
        ("src_index", C.c_void_p),
        ("aggs", C.POINTER(C.c_void_p)),
        ("form", C.c_void_p),
    ]


class hsg_stats(C.Structure):
    _fields_ = [
        ("batches", C.c_uint64),
        ("records", C.c_uint64),
        ("records_owned", C.c_uint64),
        ("pairs", C.c_uint64),
        ("late_dropped", C.c_uint64),
        ("touched", C.c_uint64),
        ("state_rows", C.c_uint64),
        ("pending_rows", C.c_uint64),
        ("last_batch_ms", C.c_double),
        ("agg_kernel_ms", C.c_double),
        ("agg_kernel_launches", C.c_uint64),
        ("exchange_ms", C.c_double),
        ("exchange_bytes", C.c_uint64),
        ("pairs_total", C.c_uint64),
        ("touched_total", C.c_uint64),
        ("state_slots", C.c_uint64),
        ("state_row_bytes", C.c_uint64),
        ("spilled_rows", C.c_uint64),
        ("spill_events", C.c_uint64),
        ("table_slots", C.c_uint64),
        ("grow_events", C.c_uint64),
        ("lean_batches", C.c_uint64),
        ("direct_batches", C.c_uint64),
        ("replays", C.c_uint64),
        ("overflow_rows", C.c_uint64),
        ("overflow_rebuilds", C.c_uint64),
    ]

    def as_dict(self):
        return {name: getattr(self, name) for name, _ in self._fields_}


# Every symbol include/hstream_gpu.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = [
    "hsg_comm_unique_id",
    "hsg_engine_create",
    "hsg_engine_destroy",
    "hsg_engine_last_error",
    "hsg_op_create",
    "hsg_op_destroy",
    "hsg_op_reset",
    "hsg_last_error",
    "hsg_push_batch",
    "hsg_push_batch_async",
    "hsg_op_wait",
    "hsg_pending_rows",
    "hsg_drain",
    "hsg_op_set_changelog",
    "hsg_state_rows",
    "hsg_dump_state",
    "hsg_op_stats",
    "hsg_testing_set_knob",
]

# testing knobs (hsg_testing_set_knob)
HSG_KNOB_XPART_LOG2 = 1
HSG_KNOB_SESS_ARENA_MIN = 2
HSG_KNOB_X_CLASSIC = 3


# Every symbol include/hstream_ingest.h declares (host ingest, no GPU needed).
INGEST_SYMBOLS = [
    "hsg_keydict_create",
    "hsg_keydict_destroy",
    "hsg_keydict_size",
    "hsg_keydict_encode",
    "hsg_keydict_text",
    "hsg_keydict_spelling_text",
    "hsg_decoder_create",
    "hsg_decoder_destroy",
    "hsg_batch_narrow",
    "hsg_decode_json_batch",
    "hsg_decode_json",
    "hsg_decode_json_spelled",
]

HSG_SPELL_ALT = 0x80000000

# hsg_decode_status
HSG_DEC_OK = 0
HSG_DEC_NOT_OBJECT = 1
HSG_DEC_NO_KEY = 2
HSG_DEC_TYPE = 3
HSG_DEC_NOT_INTEGRAL = 4
HSG_DEC_RANGE = 5


class hsg_decoder_config(C.Structure):
    _fields_ = [
        ("key_field", C.c_char_p),
        ("n_cols", C.c_int32),
        ("col_fields", C.POINTER(C.c_char_p)),
        ("col_types", C.POINTER(C.c_int32)),
        ("col_numeric", C.POINTER(C.c_uint8)),
        ("literal_forms", C.c_int32),
    ]


class hsg_sink_config(C.Structure):
    _fields_ = [
        ("windowed", C.c_int32),
        ("n_members", C.c_int32),
        ("key_field", C.c_char_p),
        ("aliases", C.POINTER(C.c_char_p)),
        ("agg_index", C.POINTER(C.c_int32)),
    ]


class hsg_sink_spellings(C.Structure):
    _fields_ = [
        ("spell", C.c_void_p),
        ("n", C.c_uint64),
        ("src_base", C.c_int64),
        ("mem", C.c_int32),
        ("reserved", C.c_int32),
    ]


class hsg_sink_records(C.Structure):
    _fields_ = [
        ("mem", C.c_int32),
        ("reserved0", C.c_int32),
        ("key_capacity", C.c_uint64),
        ("value_capacity", C.c_uint64),
        ("key_bytes", C.c_void_p),
        ("key_off", C.c_void_p),
        ("value_bytes", C.c_void_p),
        ("value_off", C.c_void_p),
    ]



# Every symbol include/hstream_sink.h declares.
SINK_SYMBOLS = ["hsg_sink_create", "hsg_sink_destroy", "hsg_sink_encode", "hsg_sink_encode_spelled",
                "hsg_sink_member_order", "hsg_format_number"]


class hsg_join_config(C.Structure):
    _fields_ = [("before_ms", C.c_int64), ("after_ms", C.c_int64), ("batch_capacity", C.c_uint64)]


class hsg_join_batch(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("mem", C.c_int32),
        ("reserved0", C.c_int32),
        ("side", C.c_void_p),
        ("key_id", C.c_void_p),
        ("join_key", C.c_void_p),
        ("ts", C.c_void_p),
        ("handle", C.c_void_p),
    ]


class hsg_join_rows(C.Structure):
    _fields_ = [
        ("capacity", C.c_uint64),
        ("mem", C.c_int32),
        ("reserved0", C.c_int32),
        ("this_handle", C.c_void_p),
        ("other_handle", C.c_void_p),
        ("join_key", C.c_void_p),
        ("ts", C.c_void_p),
    ]


# Every symbol include/hstream_join.h declares.
JOIN_SYMBOLS = ["hsg_join_create", "hsg_join_destroy", "hsg_join_last_error", "hsg_join_push", "hsg_join_pending",
                "hsg_join_drain", "hsg_join_state_rows"]


# void (*hsg_done_fn)(void *ctx, int rc)
HSG_DONE_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int)


class HStreamGpuError(RuntimeError):
    """Raised for a negative status; mirrors the reference's HStreamError (Error.hs:11-18)."""

    def __init__(self, status, message=""):
        self.status = status
        name = STATUS_NAMES.get(status, str(status))
        super().__init__(f"{name}: {message}" if message else name)


def agg_output_is_f64(kind, col_type):
    if kind in (HSG_COUNT_ALL, HSG_COUNT):
        return False
    if kind == HSG_AVG:
        return True
    return col_type == HSG_F64
