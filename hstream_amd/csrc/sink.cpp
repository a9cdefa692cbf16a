// Host side of the sink encoder (include/hstream_sink.h): fragments, the key
// texts of the ingest dictionary mirrored in HBM, scratch, and the two-pass
// encode (k_sink.hip) with an exclusive scan of the record sizes between.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/hstream_sink.h"
#include "hsg_fmt.h"
#include "hsg_sink.h"
#include "hsg_sort.h"

namespace hsg {
// hsg_api.cpp: the op's device and aggregate output types
int op_sink_info(const hsg_op *op, int *device, int *n_aggs, uint32_t *f64_mask, uint32_t *form_mask, int8_t *ident);
// ingest.cpp: the dictionary's key texts (Aeson encoding), back to back, and
// its alternate spellings
void keydict_texts(const hsg_keydict *d, const char **text, const uint64_t **off, uint64_t *n);
void keydict_alt_texts(const hsg_keydict *d, const char **text, const uint64_t **off, uint64_t *n);

static const uint64_t kPow5InvHost[HSG_POW5_INV_COUNT][2] = {HSG_POW5_INV_ROWS};
static const uint64_t kPow5Host[HSG_POW5_COUNT][2] = {HSG_POW5_ROWS};
}  // namespace hsg

using namespace hsg;

struct hsg_sink {
  int device = 0;
  hipStream_t stream = nullptr;
  SinkDev S;
  const hsg_keydict *dict = nullptr;
  int n_aggs = 0;
  char *d_frag = nullptr;
  // key texts in HBM (append-only, like the dictionary)
  char *d_ktext = nullptr;
  uint64_t ktext_cap = 0, ktext_dev = 0;
  uint64_t *d_ktoff = nullptr;
  uint64_t ktoff_cap = 0, nkeys_dev = 0;
  // alternate spellings in HBM (append-only)
  char *d_atext = nullptr;
  uint64_t atext_cap = 0, atext_dev = 0;
  uint64_t *d_atoff = nullptr;
  uint64_t atoff_cap = 0, nalt_dev = 0;
  // host rows' form / src and host spellings staged to HBM
  uint32_t *st_form = nullptr, *st_spell = nullptr;
  int64_t *st_src = nullptr;
  uint64_t st_form_cap = 0, st_spell_cap = 0, st_src_cap = 0;
  // per-row scratch
  uint64_t rows_cap = 0;
  uint32_t *klen = nullptr, *vlen = nullptr;
  uint64_t *koff = nullptr, *voff = nullptr, *partial = nullptr, *tot = nullptr;
  uint64_t *h_tot = nullptr;  // pinned [2]
  // host rows staged to HBM
  uint64_t st_cap = 0;
  uint32_t *st_key = nullptr;
  int64_t *st_ws = nullptr;
  int64_t *st_agg[kMaxAggs] = {};
  // device bytes for host destinations
  char *d_k = nullptr, *d_v = nullptr;
  uint64_t dk_cap = 0, dv_cap = 0;
};

namespace {

template <typename T>
hipError_t regrow(T *&p, uint64_t &cap, uint64_t need, bool keep = false, hipStream_t s = nullptr) {
  if (need <= cap && p) return hipSuccess;
  uint64_t nc = cap ? cap : 1024;
  while (nc < need) nc *= 2;
  T *q = nullptr;
  hipError_t e = hipMalloc((void **)&q, nc * sizeof(T));
  if (e != hipSuccess) return e;
  if (keep && p && cap) {
    e = hipMemcpyAsync(q, p, cap * sizeof(T), hipMemcpyDeviceToDevice, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      hipFree(q);
      return e;
    }
  }
  if (p) hipFree(p);
  p = q;
  cap = nc;
  return hipSuccess;
}

void put_json_string(std::string &o, const char *s) {
  static const char hx[] = "0123456789abcdef";
  o.push_back('"');
  for (const unsigned char *p = (const unsigned char *)s; *p; ++p) {
    const unsigned char ch = *p;
    if (ch == '\\') o.append("\\\\");
    else if (ch == '"') o.append("\\\"");
    else if (ch >= 0x20) o.push_back((char)ch);
    else if (ch == '\n') o.append("\\n");
    else if (ch == '\r') o.append("\\r");
    else if (ch == '\t') o.append("\\t");
    else {
      o.append("\\u00");
      o.push_back(hx[ch >> 4]);
      o.push_back(hx[ch & 15]);
    }
  }
  o.push_back('"');
}

void free_sink(hsg_sink *s) {
  if (!s) return;
  hipSetDevice(s->device);
  if (s->stream) hipStreamSynchronize(s->stream);
  void *ptrs[] = {s->d_frag, s->d_ktext, s->d_ktoff, s->klen, s->vlen, s->koff, s->voff, s->partial, s->tot,
                  s->st_key, s->st_ws, s->d_k, s->d_v, s->d_atext, s->d_atoff, s->st_form, s->st_spell, s->st_src};
  for (void *p : ptrs)
    if (p) hipFree(p);
  for (int j = 0; j < kMaxAggs; ++j)
    if (s->st_agg[j]) hipFree(s->st_agg[j]);
  if (s->h_tot) hipHostFree(s->h_tot);
  if (s->stream) hipStreamDestroy(s->stream);
  delete s;
}

#define STRY(expr)                       \
  do {                                   \
    hipError_t _e = (expr);              \
    if (_e != hipSuccess)                \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE; \
  } while (0)

// mirror the dictionary's new keys in HBM
int sync_keys(hsg_sink *s) {
  const char *text;
  const uint64_t *off;
  uint64_t n;
  keydict_texts(s->dict, &text, &off, &n);
  if (n == s->nkeys_dev) return HSG_OK;
  const uint64_t bytes = off[n];
  STRY(regrow(s->d_ktext, s->ktext_cap, bytes ? bytes : 1, true, s->stream));
  STRY(regrow(s->d_ktoff, s->ktoff_cap, n + 1, true, s->stream));
  if (bytes > s->ktext_dev)
    STRY(hipMemcpyAsync(s->d_ktext + s->ktext_dev, text + s->ktext_dev, bytes - s->ktext_dev, hipMemcpyHostToDevice,
                        s->stream));
  const uint64_t from = s->nkeys_dev ? s->nkeys_dev + 1 : 0;
  STRY(hipMemcpyAsync(s->d_ktoff + from, off + from, (n + 1 - from) * 8, hipMemcpyHostToDevice, s->stream));
  STRY(hipStreamSynchronize(s->stream));  // the dictionary's arrays may move on its next insert
  s->ktext_dev = bytes;
  s->nkeys_dev = n;
  return HSG_OK;
}

// mirror the dictionary's new alternate spellings in HBM
int sync_alts(hsg_sink *s) {
  const char *text;
  const uint64_t *off;
  uint64_t n;
  keydict_alt_texts(s->dict, &text, &off, &n);
  if (n == s->nalt_dev && s->d_atoff) return HSG_OK;
  const uint64_t bytes = off[n];
  STRY(regrow(s->d_atext, s->atext_cap, bytes ? bytes : 1, true, s->stream));
  STRY(regrow(s->d_atoff, s->atoff_cap, n + 1, true, s->stream));
  if (bytes > s->atext_dev)
    STRY(hipMemcpyAsync(s->d_atext + s->atext_dev, text + s->atext_dev, bytes - s->atext_dev, hipMemcpyHostToDevice,
                        s->stream));
  const uint64_t from = s->nalt_dev ? s->nalt_dev + 1 : 0;
  STRY(hipMemcpyAsync(s->d_atoff + from, off + from, (n + 1 - from) * 8, hipMemcpyHostToDevice, s->stream));
  STRY(hipStreamSynchronize(s->stream));
  s->atext_dev = bytes;
  s->nalt_dev = n;
  return HSG_OK;
}

// Member order of an aeson-encoded Object. aeson 1.4 writes an Object's
// members in the traversal order of its HashMap (Data.Aeson.Encoding.Internal
// dict over HM.foldrWithKey), so the sink writes them in that order too. Stack
// lts-16.21 (hstream-processing/stack.yaml:20-21; the cabal bounds
// hashable < 1.4, unordered-containers ^>= 0.2.9 in
// hstream-store/admin/hstore-admin.cabal:71,84) pins hashable-1.3.0.0,
// text-1.2.4.0 and unordered-containers-0.2.10.0:
//   hash (Text) = hashWithSalt defaultSalt: FNV-1 (prime 16777619, 64-bit)
//     over the UTF-16 code units' bytes (little-endian), seeded with
//     combine defaultSalt len = defaultSalt * 16777619 xor len,
//     defaultSalt = -2578643520546668380 (0xdc36d1615b7400a4);
//   the HAMT indexes 4-bit subkeys from the low bits (bitsPerSubkey = 4) and
//     traverses children in subkey order, so members come out in increasing
//     order of the hash read nibble by nibble from the lowest; equal hashes
//     (a collision node) keep insertion order (here: SELECT order).
// Restated from the libraries' published source; no reference test prints an
// encoded object, so the order is pinned by this restatement only
// (tests/test_sink.py restates it independently).
uint64_t aeson_key_hash(const char *utf8) {
  std::vector<uint16_t> u16;
  for (const unsigned char *p = (const unsigned char *)utf8; *p;) {
    uint32_t c = *p, extra = 0;
    if (c >= 0xF0) c &= 0x07, extra = 3;
    else if (c >= 0xE0) c &= 0x0F, extra = 2;
    else if (c >= 0xC0) c &= 0x1F, extra = 1;
    ++p;
    for (uint32_t k = 0; k < extra && (*p & 0xC0) == 0x80; ++k, ++p) c = (c << 6) | (*p & 0x3F);
    if (c >= 0x10000) {
      c -= 0x10000;
      u16.push_back((uint16_t)(0xD800 + (c >> 10)));
      u16.push_back((uint16_t)(0xDC00 + (c & 0x3FF)));
    } else {
      u16.push_back((uint16_t)c);
    }
  }
  const uint64_t prime = 16777619ull;
  uint64_t h = 0xdc36d1615b7400a4ull * prime ^ (uint64_t)u16.size();
  for (uint16_t u : u16) {
    h = (h * prime) ^ (uint64_t)(u & 0xFF);
    h = (h * prime) ^ (uint64_t)(u >> 8);
  }
  return h;
}

uint64_t nibble_reverse(uint64_t h) {
  uint64_t r = 0;
  for (int k = 0; k < 16; ++k) r = (r << 4) | ((h >> (4 * k)) & 15);
  return r;
}

}  // namespace

namespace hsg {
// for hsg_sink_member_order (tests): member m's position in the encoded object
void sink_member_order(const char *const *aliases, int n, int32_t *order) {
  std::vector<std::pair<uint64_t, int>> v;
  for (int m = 0; m < n; ++m) v.push_back({nibble_reverse(aeson_key_hash(aliases[m])), m});
  std::stable_sort(v.begin(), v.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
  for (int k = 0; k < n; ++k) order[k] = v[k].second;
}
}  // namespace hsg

extern "C" int hsg_sink_create(hsg_op *op, const hsg_keydict *dict, const hsg_sink_config *cfg, hsg_sink **out) {
  if (!op || !dict || !cfg || !out || !cfg->key_field || cfg->n_members < 0 || cfg->n_members > kSinkMaxMembers)
    return HSG_E_INVALID;
  if (cfg->n_members && (!cfg->aliases || !cfg->agg_index)) return HSG_E_INVALID;
  *out = nullptr;
  hsg_sink *s = new (std::nothrow) hsg_sink();
  if (!s) return HSG_E_OOM;
  memset(&s->S, 0, sizeof(s->S));
  uint32_t f64 = 0, fmask = 0;
  int rc = op_sink_info(op, &s->device, &s->n_aggs, &f64, &fmask, s->S.ident);
  if (rc != HSG_OK) {
    delete s;
    return rc;
  }
  for (int m = 0; m < cfg->n_members; ++m)
    if (!cfg->aliases[m] || cfg->agg_index[m] < -1 || cfg->agg_index[m] >= s->n_aggs) {
      delete s;
      return HSG_E_INVALID;
    }
  s->dict = dict;
  std::string frag;
  std::vector<uint32_t> fo;
  auto add = [&](const std::string &t) {
    fo.push_back((uint32_t)frag.size());
    frag += t;
  };
  std::string kp = "{";
  put_json_string(kp, cfg->key_field);
  kp += ":";
  add(kp);
  add("}");
  // members in the HashMap's traversal order (sink_member_order)
  int32_t order[kSinkMaxMembers];
  sink_member_order(cfg->aliases, cfg->n_members, order);
  for (int k = 0; k < cfg->n_members; ++k) {
    const int m = order[k];
    std::string t = k ? "," : "{";
    put_json_string(t, cfg->aliases[m]);
    t += ":";
    add(t);
    s->S.agg_index[k] = cfg->agg_index[m];
  }
  add(cfg->n_members ? "}" : "{}");
  fo.push_back((uint32_t)frag.size());
  for (size_t f = 0; f < fo.size(); ++f) s->S.frag_off[f] = fo[f];
  s->S.windowed = cfg->windowed ? 1 : 0;
  s->S.n_members = cfg->n_members;
  s->S.f64_mask = f64;
  s->S.form_mask = fmask;
  hipError_t e = hipSetDevice(s->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipMalloc((void **)&s->d_frag, frag.size());
  if (e == hipSuccess) e = hipMemcpy(s->d_frag, frag.data(), frag.size(), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipHostMalloc((void **)&s->h_tot, 2 * sizeof(uint64_t), hipHostMallocDefault);
  if (e == hipSuccess) e = hipMalloc((void **)&s->tot, 2 * sizeof(uint64_t));
  if (e != hipSuccess) {
    free_sink(s);
    return e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;
  }
  s->S.frag = s->d_frag;
  *out = s;
  return HSG_OK;
}

extern "C" void hsg_sink_destroy(hsg_sink *s) { free_sink(s); }

extern "C" int hsg_sink_member_order(const char *const *aliases, int32_t n, int32_t *order) {
  if (n < 0 || n > kSinkMaxMembers || (n && (!aliases || !order))) return HSG_E_INVALID;
  for (int m = 0; m < n; ++m)
    if (!aliases[m]) return HSG_E_INVALID;
  try {
    sink_member_order(aliases, n, order);
  } catch (...) {
    return HSG_E_OOM;
  }
  return HSG_OK;
}

extern "C" int hsg_sink_encode_spelled(hsg_sink *s, const hsg_rows *rows, uint64_t n, const hsg_sink_spellings *sp,
                                       hsg_sink_records *out, uint64_t *key_need, uint64_t *value_need) {
  if (!s || !rows || !out || !key_need || !value_need) return HSG_E_INVALID;
  if (sp && sp->n && (!sp->spell || !rows->src_index || (sp->mem != HSG_MEM_HOST && sp->mem != HSG_MEM_DEVICE)))
    return HSG_E_INVALID;
  if (rows->n_aggs != s->n_aggs || (rows->mem != HSG_MEM_HOST && rows->mem != HSG_MEM_DEVICE) ||
      (out->mem != HSG_MEM_HOST && out->mem != HSG_MEM_DEVICE))
    return HSG_E_INVALID;
  if (n && (!rows->key_id || (s->S.windowed && !rows->win_start))) return HSG_E_INVALID;
  bool need_agg[kMaxAggs] = {};
  for (int m = 0; m < s->S.n_members; ++m)
    if (s->S.agg_index[m] >= 0) {
      need_agg[s->S.agg_index[m]] = true;
      if (n && (!rows->aggs || !rows->aggs[s->S.agg_index[m]])) return HSG_E_INVALID;
    }
  if (!out->key_off || !out->value_off) return HSG_E_INVALID;
  try {
    STRY(hipSetDevice(s->device));
    int rc = sync_keys(s);
    if (rc == HSG_OK) rc = sync_alts(s);
    if (rc != HSG_OK) return rc;
    hipStream_t st = s->stream;
    *key_need = *value_need = 0;
    if (n == 0) {
      const uint64_t z = 0;
      if (out->mem == HSG_MEM_HOST) {
        out->key_off[0] = out->value_off[0] = 0;
      } else {
        STRY(hipMemcpy(out->key_off, &z, 8, hipMemcpyHostToDevice));
        STRY(hipMemcpy(out->value_off, &z, 8, hipMemcpyHostToDevice));
      }
      return HSG_OK;
    }
    SinkDev S = s->S;
    S.ktext = s->d_ktext;
    S.ktoff = s->d_ktoff;
    S.nkeys = s->nkeys_dev;
    S.atext = s->d_atext;
    S.atoff = s->d_atoff;
    S.nalt = s->nalt_dev;
    // literal forms and record spellings: device pointers (host arrays staged)
    const bool hrows = rows->mem == HSG_MEM_HOST;
    if (rows->form && s->S.form_mask) {
      if (hrows) {
        STRY(regrow(s->st_form, s->st_form_cap, n));
        STRY(hipMemcpyAsync(s->st_form, rows->form, n * 4, hipMemcpyHostToDevice, st));
        S.form = s->st_form;
      } else {
        S.form = rows->form;
      }
    }
    if (sp && sp->n) {
      if (hrows) {
        STRY(regrow(s->st_src, s->st_src_cap, n));
        STRY(hipMemcpyAsync(s->st_src, rows->src_index, n * 8, hipMemcpyHostToDevice, st));
        S.src = s->st_src;
      } else {
        S.src = rows->src_index;
      }
      if (sp->mem == HSG_MEM_HOST) {
        STRY(regrow(s->st_spell, s->st_spell_cap, sp->n));
        STRY(hipMemcpyAsync(s->st_spell, sp->spell, sp->n * 4, hipMemcpyHostToDevice, st));
        S.spell = s->st_spell;
      } else {
        S.spell = sp->spell;
      }
      S.src_base = sp->src_base;
      S.nspell = sp->n;
    }
    if (rows->mem == HSG_MEM_DEVICE) {
      S.key = rows->key_id;
      S.ws = rows->win_start;
      for (int j = 0; j < s->n_aggs; ++j) S.agg[j] = need_agg[j] ? (const int64_t *)rows->aggs[j] : nullptr;
    } else {
      if (n > s->st_cap) {
        uint64_t c = 0;
        STRY(regrow(s->st_key, c, n));
        c = 0;
        STRY(regrow(s->st_ws, c, n));
        for (int j = 0; j < s->n_aggs; ++j) {
          c = 0;
          STRY(regrow(s->st_agg[j], c, n));
        }
        s->st_cap = c;
      }
      STRY(hipMemcpyAsync(s->st_key, rows->key_id, n * 4, hipMemcpyHostToDevice, st));
      if (s->S.windowed) STRY(hipMemcpyAsync(s->st_ws, rows->win_start, n * 8, hipMemcpyHostToDevice, st));
      for (int j = 0; j < s->n_aggs; ++j)
        if (need_agg[j]) STRY(hipMemcpyAsync(s->st_agg[j], rows->aggs[j], n * 8, hipMemcpyHostToDevice, st));
      S.key = s->st_key;
      S.ws = s->st_ws;
      for (int j = 0; j < s->n_aggs; ++j) S.agg[j] = need_agg[j] ? s->st_agg[j] : nullptr;
    }
    if (n > s->rows_cap) {
      uint64_t c = 0;
      STRY(regrow(s->klen, c, n));
      c = 0;
      STRY(regrow(s->vlen, c, n));
      c = 0;
      STRY(regrow(s->koff, c, n + 1));
      c = 0;
      STRY(regrow(s->voff, c, n + 1));
      c = 0;
      STRY(regrow(s->partial, c, scan_partials_needed(n) + 8));
      s->rows_cap = n;
    }
    launch_sink_len(st, S, n, s->klen, s->vlen);
    scan_excl_u32(st, s->klen, s->koff, n, s->partial, s->tot);
    scan_excl_u32(st, s->vlen, s->voff, n, s->partial, s->tot + 1);
    STRY(hipMemcpyAsync(s->h_tot, s->tot, 16, hipMemcpyDeviceToHost, st));
    STRY(hipStreamSynchronize(st));
    STRY(hipGetLastError());
    const uint64_t kb = s->h_tot[0], vb = s->h_tot[1];
    *key_need = kb;
    *value_need = vb;
    if (kb > out->key_capacity || vb > out->value_capacity) return HSG_E_CAPACITY;
    if (!out->key_bytes || !out->value_bytes) return HSG_E_INVALID;
    // offsets[n] = totals
    STRY(hipMemcpyAsync(s->koff + n, s->tot, 8, hipMemcpyDeviceToDevice, st));
    STRY(hipMemcpyAsync(s->voff + n, s->tot + 1, 8, hipMemcpyDeviceToDevice, st));
    if (out->mem == HSG_MEM_DEVICE) {
      launch_sink_write(st, S, n, s->koff, s->voff, out->key_bytes, out->value_bytes);
      STRY(hipMemcpyAsync(out->key_off, s->koff, (n + 1) * 8, hipMemcpyDeviceToDevice, st));
      STRY(hipMemcpyAsync(out->value_off, s->voff, (n + 1) * 8, hipMemcpyDeviceToDevice, st));
    } else {
      STRY(regrow(s->d_k, s->dk_cap, kb ? kb : 1));
      STRY(regrow(s->d_v, s->dv_cap, vb ? vb : 1));
      launch_sink_write(st, S, n, s->koff, s->voff, s->d_k, s->d_v);
      STRY(hipMemcpyAsync(out->key_bytes, s->d_k, kb, hipMemcpyDeviceToHost, st));
      STRY(hipMemcpyAsync(out->value_bytes, s->d_v, vb, hipMemcpyDeviceToHost, st));
      STRY(hipMemcpyAsync(out->key_off, s->koff, (n + 1) * 8, hipMemcpyDeviceToHost, st));
      STRY(hipMemcpyAsync(out->value_off, s->voff, (n + 1) * 8, hipMemcpyDeviceToHost, st));
    }
    STRY(hipStreamSynchronize(st));
    STRY(hipGetLastError());
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  }
}

extern "C" int hsg_sink_encode(hsg_sink *s, const hsg_rows *rows, uint64_t n, hsg_sink_records *out,
                               uint64_t *key_need, uint64_t *value_need) {
  return hsg_sink_encode_spelled(s, rows, n, nullptr, out, key_need, value_need);
}

extern "C" int hsg_format_number(int32_t is_f64, int64_t bits, char *buf, size_t cap, size_t *len) {
  if (!len) return HSG_E_INVALID;
  char t[kNumTextMax];
  int n;
  if (is_f64) {
    const Pow5Tables T{kPow5InvHost, kPow5Host};
    double v;
    memcpy(&v, &bits, 8);
    n = fmt_f64(v, T, t, is_f64 >= 2 ? is_f64 - 2 : -1);
  } else {
    n = fmt_i64(bits, t);
  }
  *len = (size_t)n;
  if (cap < (size_t)n || !buf) return HSG_E_CAPACITY;
  memcpy(buf, t, (size_t)n);
  return HSG_OK;
}
