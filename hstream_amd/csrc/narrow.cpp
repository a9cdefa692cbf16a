// Host side of the narrow transport (include/hstream_gpu.h hsg_enc): a
// decoded poll batch is rewritten in place into the narrowest encoding that
// is lossless for the values it holds, so it crosses PCIe in fewer bytes; the
// library widens it on the device before any kernel sees it. The decoder
// (hsg_decode_json_batch, ingest.cpp) calls it on every batch it decodes.
//
// What is chosen (each only when the consumer allows it, HSG_NARROW_*):
//   key  K16    every key id < 2^16 (no HSG_KEY_NONE record)
//   ts   TS16   every frame of HSG_TS16_FRAME records spans < 2^16 ms: uint16
//               offsets from the frame's minimum, else
//        TS32   the batch spans < 2^31 ms: int32 offsets from its minimum
//   i64  I32    every value (absent ones are 0) fits int32
//   f64  DEC32  one scale s <= 9 with every value v = m / 10^s exactly (the
//               double the device's division gives back), |m| < 2^31, and no
//               -0.0 (a mantissa has no sign for zero)
// The statistics run over host threads; the rewrite is one forward pass per
// column (a narrower element never overtakes the wider one it replaces).
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/hstream_gpu.h"
#include "../../include/hstream_ingest.h"

namespace {

constexpr int kNoScale = 99;
constexpr int kMaxScale = 9;
const double kP10[kMaxScale + 1] = {1e0, 1e1, 1e2, 1e3, 1e4, 1e5, 1e6, 1e7, 1e8, 1e9};

// smallest s with v == m / 10^s for an integer |m| < 2^31, else kNoScale
int dec_scale(double v) {
  if (v == 0.0) return std::signbit(v) ? kNoScale : 0;
  if (!std::isfinite(v)) return kNoScale;
  for (int s = 0; s <= kMaxScale; ++s) {
    const double m = std::nearbyint(v * kP10[s]);
    if (std::fabs(m) >= 2147483648.0) return kNoScale;
    if (m / kP10[s] == v) return s;
  }
  return kNoScale;
}

bool dec_fits(double v, int s) {
  if (v == 0.0) return !std::signbit(v);
  const double m = std::nearbyint(v * kP10[s]);
  return std::fabs(m) < 2147483648.0 && m / kP10[s] == v;
}

struct Stats {
  uint32_t kmax = 0;
  int64_t tmin = INT64_MAX, tmax = INT64_MIN;
  bool ts16 = true;
  int64_t cmin[8], cmax[8];
  int scale[8];
  bool present[8];  // every record present, no literal-form bit
};

}  // namespace

extern "C" int hsg_batch_narrow(hsg_batch *io, const int32_t *col_types, uint32_t allow, int64_t *ts_frames,
                                uint32_t *present_mask, int n_threads) {
  if (present_mask) *present_mask = 0;
  if (!io || io->mem != HSG_MEM_HOST || io->n_cols < 0 || io->n_cols > 8) return HSG_E_INVALID;
  if (io->n_cols && !col_types) return HSG_E_INVALID;
  if (io->ts_enc != HSG_ENC_FULL || io->key_enc != HSG_ENC_FULL) return HSG_E_INVALID;
  for (int c = 0; c < io->n_cols; ++c)
    if (io->col_enc[c] != HSG_ENC_FULL) return HSG_E_INVALID;
  const uint64_t n = io->n;
  const int C = io->n_cols;
  if (!n) return HSG_OK;
  if ((allow & HSG_NARROW_TS16) && !ts_frames) allow &= ~HSG_NARROW_TS16;
  uint32_t *key = (uint32_t *)io->key_id;
  int64_t *ts = (int64_t *)io->ts;
  const uint64_t F = (n + HSG_TS16_FRAME - 1) / HSG_TS16_FRAME;
  try {
    int T = n_threads > 0 ? n_threads : (int)std::thread::hardware_concurrency();
    if (T < 1) T = 1;
    if (T > 32) T = 32;
    if ((uint64_t)T > F) T = (int)F;
    std::vector<Stats> st((size_t)T);
    auto work = [&](int t) {
      Stats &s = st[(size_t)t];
      for (int c = 0; c < C; ++c) {
        s.cmin[c] = INT64_MAX;
        s.cmax[c] = INT64_MIN;
        s.scale[c] = 0;
        s.present[c] = true;
      }
      const uint64_t f0 = F * (uint64_t)t / (uint64_t)T, f1 = F * (uint64_t)(t + 1) / (uint64_t)T;
      for (uint64_t f = f0; f < f1; ++f) {
        const uint64_t lo = f * HSG_TS16_FRAME, hi = lo + HSG_TS16_FRAME < n ? lo + HSG_TS16_FRAME : n;
        int64_t fmin = INT64_MAX, fmax = INT64_MIN;
        for (uint64_t i = lo; i < hi; ++i) {
          s.kmax = key[i] > s.kmax ? key[i] : s.kmax;
          fmin = ts[i] < fmin ? ts[i] : fmin;
          fmax = ts[i] > fmax ? ts[i] : fmax;
        }
        if (ts_frames) ts_frames[f] = fmin;
        s.ts16 = s.ts16 && (uint64_t)fmax - (uint64_t)fmin < 65536u;
        s.tmin = fmin < s.tmin ? fmin : s.tmin;
        s.tmax = fmax > s.tmax ? fmax : s.tmax;
        for (int c = 0; c < C; ++c) {
          const uint8_t *v = io->valid ? io->valid[c] : nullptr;
          if (v)
            for (uint64_t i = lo; i < hi && s.present[c]; ++i) s.present[c] = v[i] == 1;
          if (col_types[c] == HSG_I64) {
            const int64_t *x = (const int64_t *)io->cols[c];
            for (uint64_t i = lo; i < hi; ++i) {
              s.cmin[c] = x[i] < s.cmin[c] ? x[i] : s.cmin[c];
              s.cmax[c] = x[i] > s.cmax[c] ? x[i] : s.cmax[c];
            }
          } else if (s.scale[c] != kNoScale) {
            const double *x = (const double *)io->cols[c];
            for (uint64_t i = lo; i < hi; ++i) {
              const int k = dec_scale(x[i]);
              if (k > s.scale[c]) {
                s.scale[c] = k;
                if (k == kNoScale) break;
              }
            }
          }
        }
      }
    };
    if (T == 1) {
      work(0);
    } else {
      std::vector<std::thread> th;
      for (int t = 1; t < T; ++t) th.emplace_back(work, t);
      work(0);
      for (auto &x : th) x.join();
    }
    Stats all = st[0];
    for (int t = 1; t < T; ++t) {
      const Stats &s = st[(size_t)t];
      all.kmax = s.kmax > all.kmax ? s.kmax : all.kmax;
      all.tmin = s.tmin < all.tmin ? s.tmin : all.tmin;
      all.tmax = s.tmax > all.tmax ? s.tmax : all.tmax;
      all.ts16 = all.ts16 && s.ts16;
      for (int c = 0; c < C; ++c) {
        all.cmin[c] = s.cmin[c] < all.cmin[c] ? s.cmin[c] : all.cmin[c];
        all.cmax[c] = s.cmax[c] > all.cmax[c] ? s.cmax[c] : all.cmax[c];
        all.scale[c] = s.scale[c] > all.scale[c] ? s.scale[c] : all.scale[c];
        all.present[c] = all.present[c] && s.present[c];
      }
    }
    if (present_mask)
      for (int c = 0; c < C; ++c) *present_mask |= all.present[c] ? 1u << c : 0u;
    // key ids
    if ((allow & HSG_NARROW_K16) && all.kmax < 65536u) {
      uint16_t *k16 = (uint16_t *)key;
      for (uint64_t i = 0; i < n; ++i) k16[i] = (uint16_t)key[i];
      io->key_enc = HSG_ENC_K16;
    }
    // timestamps
    if ((allow & HSG_NARROW_TS16) && all.ts16) {
      uint16_t *t16 = (uint16_t *)ts;
      for (uint64_t i = 0; i < n; ++i) t16[i] = (uint16_t)((uint64_t)ts[i] - (uint64_t)ts_frames[i / HSG_TS16_FRAME]);
      io->ts_enc = HSG_ENC_TS16;
      io->ts_frames = ts_frames;
    } else if ((allow & HSG_NARROW_TS32) && (uint64_t)all.tmax - (uint64_t)all.tmin < 0x80000000ull) {
      int32_t *t32 = (int32_t *)ts;
      for (uint64_t i = 0; i < n; ++i) t32[i] = (int32_t)((uint64_t)ts[i] - (uint64_t)all.tmin);
      io->ts_enc = HSG_ENC_TS32;
      io->ts_base = all.tmin;
    }
    // value columns
    for (int c = 0; c < C; ++c) {
      void *col = (void *)io->cols[c];
      if (col_types[c] == HSG_I64) {
        if (!(allow & HSG_NARROW_I32) || all.cmin[c] < INT32_MIN || all.cmax[c] > INT32_MAX) continue;
        const int64_t *x = (const int64_t *)col;
        int32_t *y = (int32_t *)col;
        for (uint64_t i = 0; i < n; ++i) y[i] = (int32_t)x[i];
        io->col_enc[c] = HSG_ENC_I32;
      } else {
        const int s = all.scale[c];
        if (!(allow & HSG_NARROW_DEC32) || s == kNoScale) continue;
        const double *x = (const double *)col;
        bool ok = true;  // a value exact at its own scale is exact at a larger one unless |m| outgrows int32
        for (uint64_t i = 0; i < n && ok; ++i) ok = dec_fits(x[i], s);
        if (!ok) continue;
        int32_t *y = (int32_t *)col;
        for (uint64_t i = 0; i < n; ++i) y[i] = (int32_t)std::nearbyint(x[i] * kP10[s]);
        io->col_enc[c] = HSG_ENC_DEC32;
        io->col_scale[c] = (uint8_t)s;
      }
    }
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  } catch (...) {
    return HSG_E_INVALID;
  }
}

