"""Host side of the narrow transport (include/hstream_gpu.h hsg_enc): what a
producer may send narrower, and that a DEC32 value is exactly the double its
decimal text parses to (the device computes m / 10^s the same way)."""
import numpy as np

from hstream_amd import abi
from hstream_amd.columnar import make_batch, narrow_columns


def test_dec32_is_the_parsed_double():
    rng = np.random.default_rng(3)
    m = rng.integers(-2**31, 2**31, 3000)
    for s in (0, 1, 3, 6, 9):
        def text(x):
            a = abs(int(x))
            return ("-" if x < 0 else "") + (f"{a // 10**s}.{a % 10**s:0{s}d}" if s else str(a))
        parsed = np.array([float(text(x)) for x in m])
        assert np.array_equal(m / 10.0**s, parsed), s


def test_narrow_columns_choices():
    ts = np.array([1_700_000_000_000, 1_700_000_000_500, 1_699_999_999_000], np.int64)
    i64 = np.array([-5, 2**31 - 1, -2**31], np.int64)
    big = np.array([0, 2**31], np.int64)
    f = np.array([1.5, 2.25, 123456.789], np.float64)
    t32, base, cs, enc, scale = narrow_columns(ts, [i64, big, f, f], [abi.HSG_I64, abi.HSG_I64, abi.HSG_F64,
                                                                      abi.HSG_F64], [None, None, 3, 2])
    assert base == 1_699_999_999_000 and t32.dtype == np.int32
    assert np.array_equal(base + t32.astype(np.int64), ts)
    assert enc == [abi.HSG_ENC_I32, abi.HSG_ENC_FULL, abi.HSG_ENC_DEC32, abi.HSG_ENC_FULL], enc
    assert scale[2] == 3 and np.array_equal(cs[2] / 1e3, f)
    # a ts span of 2^31 ms or more stays full width
    _, base2, _, _, _ = narrow_columns(np.array([0, 2**31], np.int64), [], [])
    assert base2 is None


def test_make_batch_fields():
    key = np.arange(4, dtype=np.uint32)
    b, _ = make_batch(key, np.arange(4, dtype=np.int32), [np.arange(4, dtype=np.int32)], None, abi.HSG_MEM_HOST,
                      ts_base=77, col_enc=[abi.HSG_ENC_I32], col_scale=[0])
    assert b.ts_enc == abi.HSG_ENC_TS32 and b.ts_base == 77 and b.col_enc[0] == abi.HSG_ENC_I32
    b2, _ = make_batch(key, np.arange(4, dtype=np.int64), [np.arange(4, dtype=np.int64)], None, abi.HSG_MEM_HOST)
    assert b2.ts_enc == abi.HSG_ENC_FULL and b2.col_enc[0] == abi.HSG_ENC_FULL


def test_ts16_frames():
    from hstream_amd.columnar import narrow_ts16
    rng = np.random.default_rng(5)
    n = 3 * abi.HSG_TS16_FRAME + 17
    ts = 1_700_000_000_000 + np.arange(n) * 3 + rng.integers(0, 2000, n)
    off, fr = narrow_ts16(ts)
    assert off.dtype == np.uint16 and fr.size == 4
    assert np.array_equal(np.repeat(fr, abi.HSG_TS16_FRAME)[:n] + off.astype(np.int64), ts)
    # a frame spanning 65536 ms or more: not TS16 (narrow_columns falls back to TS32)
    ts2 = ts.copy()
    ts2[5] += 70_000
    assert narrow_ts16(ts2) is None
    t, base, _, _, _ = narrow_columns(ts2, [], [], ts16=True)
    assert t.dtype == np.int32 and isinstance(base, int)
    t, fr2, _, _, _ = narrow_columns(ts, [], [], ts16=True)
    assert t.dtype == np.uint16 and np.array_equal(fr2, fr)
    b, _ = make_batch(np.arange(n, dtype=np.uint32), off, [], None, abi.HSG_MEM_HOST, ts_frames=fr)
    assert b.ts_enc == abi.HSG_ENC_TS16 and b.ts_frames


def test_dec32_keeps_signed_zero_full_width():
    """-0.0 equals 0.0 numerically but a DEC32 mantissa 0 widens to +0.0: a
    column holding -0.0 is not lossless as DEC32 and stays full width."""
    f = np.array([1.5, -0.0, 2.25], np.float64)
    _, _, cs, enc, _ = narrow_columns(np.zeros(3, np.int64), [f], [abi.HSG_F64], [2])
    assert enc == [abi.HSG_ENC_FULL] and np.signbit(cs[0][1])
    g = np.array([1.5, 0.0, 2.25], np.float64)
    _, _, _, enc, _ = narrow_columns(np.zeros(3, np.int64), [g], [abi.HSG_F64], [2])
    assert enc == [abi.HSG_ENC_DEC32]
