// Number text of the sink encoder, the same on the host and the device:
// aggregates printed the way the reference's sink prints them (aeson-1.4
// `encode` of an Object whose values are Data.Scientific numbers).
//   * int64 values (COUNT, integer SUM/MIN/MAX/LAST) are Scientifics with
//     exponent 0, which aeson prints as plain integers.
//   * f64 values (AVG, decimal SUM/MIN/MAX) print through Scientific's
//     formatScientific Generic (what aeson uses for exponents < 0): the shortest
//     decimal that reads back as the same double (Ryu: Ulf Adams, "Ryu: fast
//     float-to-string conversion", PLDI 2018), in fixed notation for
//     0.1 <= |x| < 10^7 ("1234.5", "4.0", "0.25"), else d.ddd e n ("1.0e-3").
//     The reference's decimals are exact; an f64 sum that is not is printed
//     as the decimal of the double it is.
// Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "hsg_ryu_tables.h"

namespace hsg {

#define HSG_HD __host__ __device__ inline

struct Pow5Tables {
  const uint64_t (*inv)[2];  // HSG_POW5_INV_ROWS
  const uint64_t (*pow)[2];  // HSG_POW5_ROWS
};

// longest text of one number (sign + 20 digits, or d.ddddddddddddddddde-324)
constexpr int kNumTextMax = 32;
// an integral f64 printed as an integer (literal forms): up to 309 digits
constexpr int kNumTextIntMax = 328;

HSG_HD int fmt_u64_digits(uint64_t v, char *out) {
  char t[20];
  int n = 0;
  do {
    t[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  for (int i = 0; i < n; ++i) out[i] = t[n - 1 - i];
  return n;
}

HSG_HD int fmt_i64(int64_t v, char *out) {
  if (v < 0) {
    out[0] = '-';
    return 1 + fmt_u64_digits((uint64_t)0 - (uint64_t)v, out + 1);
  }
  return fmt_u64_digits((uint64_t)v, out);
}

// Scientific Generic text of neg * D * 10^e (D = nd digits, no trailing zero;
// nd == 0 means zero)
HSG_HD int fmt_generic(bool neg, const char *d, int nd, int e, char *out) {
  int k = 0;
  if (nd == 0) {
    out[0] = '0', out[1] = '.', out[2] = '0';
    return 3;
  }
  if (neg) out[k++] = '-';
  const int E = nd + e;  // value = 0.D * 10^E
  if (E < 0 || E > 7) {
    out[k++] = d[0];
    out[k++] = '.';
    if (nd > 1) {
      for (int i = 1; i < nd; ++i) out[k++] = d[i];
    } else {
      out[k++] = '0';
    }
    out[k++] = 'e';
    k += fmt_i64(E - 1, out + k);
    return k;
  }
  if (E == 0) {
    out[k++] = '0';
    out[k++] = '.';
    for (int i = 0; i < nd; ++i) out[k++] = d[i];
    return k;
  }
  for (int i = 0; i < E; ++i) out[k++] = i < nd ? d[i] : '0';
  out[k++] = '.';
  if (nd > E) {
    for (int i = E; i < nd; ++i) out[k++] = d[i];
  } else {
    out[k++] = '0';
  }
  return k;
}

// ---- Ryu d2d ---------------------------------------------------------------
HSG_HD uint32_t ryu_pow5bits(int32_t e) { return (uint32_t)(((uint32_t)e * 1217359u) >> 19) + 1; }
HSG_HD uint32_t ryu_log10pow2(int32_t e) { return ((uint32_t)e * 78913u) >> 18; }
HSG_HD uint32_t ryu_log10pow5(int32_t e) { return ((uint32_t)e * 732923u) >> 20; }

HSG_HD uint32_t ryu_pow5factor(uint64_t v) {
  uint32_t c = 0;
  while (v && v % 5 == 0) {
    v /= 5;
    ++c;
  }
  return c;
}
HSG_HD bool ryu_multiple_of_pow5(uint64_t v, uint32_t p) { return ryu_pow5factor(v) >= p; }
HSG_HD bool ryu_multiple_of_pow2(uint64_t v, uint32_t p) { return (v & ((1ull << p) - 1)) == 0; }

// (m * mul) >> j for a 125-bit mul and j >= 64
HSG_HD uint64_t ryu_mulshift(uint64_t m, const uint64_t *mul, int32_t j) {
  const unsigned __int128 b0 = (unsigned __int128)m * mul[0];
  const unsigned __int128 b2 = (unsigned __int128)m * mul[1];
  return (uint64_t)(((b0 >> 64) + b2) >> (j - 64));
}

// shortest decimal of a finite, nonzero double: value = out * 10^e10
HSG_HD void ryu_d2d(uint64_t ieee_m, uint32_t ieee_e, const Pow5Tables &T, uint64_t &out, int32_t &e10_out) {
  int32_t e2;
  uint64_t m2;
  if (ieee_e == 0) {
    e2 = 1 - 1023 - 52 - 2;
    m2 = ieee_m;
  } else {
    e2 = (int32_t)ieee_e - 1023 - 52 - 2;
    m2 = (1ull << 52) | ieee_m;
  }
  const bool even = (m2 & 1) == 0;
  const bool accept = even;
  const uint64_t mv = 4 * m2;
  const uint32_t mm_shift = (ieee_m != 0 || ieee_e <= 1) ? 1u : 0u;
  uint64_t vr, vp, vm;
  int32_t e10;
  bool vm_tz = false, vr_tz = false;
  if (e2 >= 0) {
    const uint32_t q = ryu_log10pow2(e2) - (e2 > 3 ? 1u : 0u);
    e10 = (int32_t)q;
    const int32_t k = HSG_POW5_INV_BITS + (int32_t)ryu_pow5bits((int32_t)q) - 1;
    const int32_t i = -e2 + (int32_t)q + k;
    vr = ryu_mulshift(4 * m2, T.inv[q], i);
    vp = ryu_mulshift(4 * m2 + 2, T.inv[q], i);
    vm = ryu_mulshift(4 * m2 - 1 - mm_shift, T.inv[q], i);
    if (q <= 21) {
      const uint32_t mv_mod5 = (uint32_t)(mv % 5);
      if (mv_mod5 == 0) vr_tz = ryu_multiple_of_pow5(mv, q);
      else if (accept) vm_tz = ryu_multiple_of_pow5(mv - 1 - mm_shift, q);
      else vp -= ryu_multiple_of_pow5(mv + 2, q) ? 1 : 0;
    }
  } else {
    const uint32_t q = ryu_log10pow5(-e2) - (-e2 > 1 ? 1u : 0u);
    e10 = (int32_t)q + e2;
    const int32_t i = -e2 - (int32_t)q;
    const int32_t k = (int32_t)ryu_pow5bits(i) - HSG_POW5_BITS;
    const int32_t j = (int32_t)q - k;
    vr = ryu_mulshift(4 * m2, T.pow[i], j);
    vp = ryu_mulshift(4 * m2 + 2, T.pow[i], j);
    vm = ryu_mulshift(4 * m2 - 1 - mm_shift, T.pow[i], j);
    if (q <= 1) {
      vr_tz = true;
      if (accept) vm_tz = mm_shift == 1;
      else --vp;
    } else if (q < 63) {
      vr_tz = ryu_multiple_of_pow2(mv, q);
    }
  }
  int32_t removed = 0;
  uint8_t last = 0;
  uint64_t output;
  if (vm_tz || vr_tz) {
    while (vp / 10 > vm / 10) {
      vm_tz &= vm % 10 == 0;
      vr_tz &= last == 0;
      last = (uint8_t)(vr % 10);
      vr /= 10;
      vp /= 10;
      vm /= 10;
      ++removed;
    }
    if (vm_tz) {
      while (vm % 10 == 0) {
        vr_tz &= last == 0;
        last = (uint8_t)(vr % 10);
        vr /= 10;
        vp /= 10;
        vm /= 10;
        ++removed;
      }
    }
    if (vr_tz && last == 5 && vr % 2 == 0) last = 4;  // ties to even
    output = vr + (((vr == vm && (!accept || !vm_tz)) || last >= 5) ? 1 : 0);
  } else {
    bool round_up = false;
    while (vp / 10 > vm / 10) {
      round_up = vr % 10 >= 5;
      vr /= 10;
      vp /= 10;
      vm /= 10;
      ++removed;
    }
    output = vr + ((vr == vm || round_up) ? 1 : 0);
  }
  out = output;
  e10_out = e10 + removed;
}

// f64 -> aeson text; returns the length (<= kNumTextMax). ident: the kind of
// aggregate the value is, for rows without literal forms (with them the sink
// knows which rows are identities): 0 SUM, 1 MIN, 2 MAX map that aggregate's
// identity to the reference's integer initial value; -1 prints exactly.
HSG_HD int fmt_f64(double v, const Pow5Tables &T, char *out, int ident = -1) {
  uint64_t bits;
  memcpy(&bits, &v, 8);
  const bool neg = (bits >> 63) != 0;
  const uint32_t ie = (uint32_t)((bits >> 52) & 0x7FF);
  const uint64_t im = bits & ((1ull << 52) - 1);
  if (ie == 0x7FF) {  // no Scientific is NaN or infinite; aeson's Double encoding prints null
    out[0] = 'n', out[1] = 'u', out[2] = 'l', out[3] = 'l';
    return 4;
  }
  // Aggregate identities are integers in the reference (Codegen.hs:425,438,
  // 451: Number 0, minBound / maxBound :: Int, exponent 0), which aeson prints
  // plainly. Here a SUM no value reached keeps its identity -0.0
  // (slot_identity), a MIN / MAX the f64 image of maxBound (2^63, rounded) /
  // minBound (-2^63).
  if (ident == 0 && bits == 0x8000000000000000ull) {
    out[0] = '0';
    return 1;
  }
  if (ident == 1 && v == 9223372036854775808.0) return fmt_i64(INT64_MAX, out);
  if (ident == 2 && v == -9223372036854775808.0) return fmt_i64(INT64_MIN, out);
  if (ie == 0 && im == 0) return fmt_generic(false, nullptr, 0, 0, out);
  uint64_t m;
  int32_t e;
  ryu_d2d(im, ie, T, m, e);
  while (m % 10 == 0) {
    m /= 10;
    ++e;
  }
  char d[20];
  const int nd = fmt_u64_digits(m, d);
  return fmt_generic(neg, d, nd, e, out);
}

// An int64 whose Scientific has a negative exponent (a sum of decimal
// literals that came out integral, "6.0"): Scientific's Generic form.
HSG_HD int fmt_i64_decimal(int64_t v, char *out) {
  if (v == 0) return fmt_generic(false, nullptr, 0, 0, out);
  uint64_t m = v < 0 ? (uint64_t)0 - (uint64_t)v : (uint64_t)v;
  int e = 0;
  while (m % 10 == 0) {
    m /= 10;
    ++e;
  }
  char d[20];
  const int nd = fmt_u64_digits(m, d);
  return fmt_generic(v < 0, d, nd, e, out);
}

// An integral f64 whose Scientific has an exponent >= 0 (a sum of integer
// literals, "6"): the integer; below 2^63 exactly, above it the shortest
// round-trip digits followed by zeros (the f64 holds no more). <= kNumTextIntMax.
HSG_HD int fmt_f64_integral(double v, const Pow5Tables &T, char *out) {
  if (v > -9223372036854775808.0 && v < 9223372036854775808.0) return fmt_i64((int64_t)v, out);
  uint64_t bits;
  memcpy(&bits, &v, 8);
  const uint32_t ie = (uint32_t)((bits >> 52) & 0x7FF);
  if (ie == 0x7FF) return fmt_f64(v, T, out);
  uint64_t m;
  int32_t e;
  ryu_d2d(bits & ((1ull << 52) - 1), ie, T, m, e);
  int k = 0;
  if (bits >> 63) out[k++] = '-';
  k += fmt_u64_digits(m, out + k);
  for (int32_t q = 0; q < e && k < kNumTextIntMax; ++q) out[k++] = '0';
  return k;
}

#undef HSG_HD

}  // namespace hsg
