// gfx950 sink encoder: changelog rows -> the key / value bytes the
// reference's sink serdes produce (include/hstream_sink.h). Two passes over
// the rows, one thread per row: byte counts, an exclusive scan (sink.cpp),
// then every record written at its offset. Numbers are formatted in
// registers (hsg_fmt.h); the Ryu tables live in constant memory.
#include "hsg_dev.h"
#include "hsg_fmt.h"
#include "hsg_sink.h"

namespace hsg {

static __constant__ uint64_t kPow5InvDev[HSG_POW5_INV_COUNT][2] = {HSG_POW5_INV_ROWS};
static __constant__ uint64_t kPow5Dev[HSG_POW5_COUNT][2] = {HSG_POW5_ROWS};

__device__ inline uint32_t frag_len(const SinkDev &S, int f) { return S.frag_off[f + 1] - S.frag_off[f]; }

__device__ inline void key_text(const SinkDev &S, uint32_t k, const char *&p, uint32_t &n) {
  if ((k & HSG_SPELL_ALT) && k != HSG_KEY_NONE && (uint64_t)(k & ~HSG_SPELL_ALT) < S.nalt) {
    const uint32_t a = k & ~HSG_SPELL_ALT;
    p = S.atext + S.atoff[a];
    n = (uint32_t)(S.atoff[a + 1] - S.atoff[a]);
  } else if (k < S.nkeys) {
    p = S.ktext + S.ktoff[k];
    n = (uint32_t)(S.ktoff[k + 1] - S.ktoff[k]);
  } else {  // HSG_KEY_NONE never reaches a changelog; an unknown id prints as null
    p = "null";
    n = 4;
  }
}

// the text a row's key prints with: its record's own spelling when the rows
// carry their source records and the batch's spellings are given (the
// reference forwards each record with its own key, TimeWindowedStream.hs:94,101),
// else the key's first spelling
__device__ inline uint32_t row_key(const SinkDev &S, uint64_t i) {
  const uint32_t k = S.key[i];
  if (S.spell && S.src) {
    const int64_t r = S.src[i] - S.src_base;
    if (r >= 0 && (uint64_t)r < S.nspell) {
      const uint32_t sp = S.spell[r];
      if (sp != HSG_KEY_NONE) return sp;
    }
  }
  return k;
}

// text of value member m of row i into buf (numbers) or as a pointer (key text).
// FORMS: the op kept literal forms (an integral f64 may print all its digits,
// up to kNumTextIntMax bytes); else every number fits kNumTextMax, so the
// default kernels keep a 32-byte buffer per thread instead of a 328-byte one
template <bool FORMS>
__device__ inline uint32_t member_text(const SinkDev &S, int m, uint64_t i, uint32_t k, char *buf, const char *&p) {
  const int j = S.agg_index[m];
  if (j < 0) {
    uint32_t n;
    key_text(S, k, p, n);
    return n;
  }
  p = buf;
  const int64_t v = S.agg[j][i];
  const bool f64 = (S.f64_mask >> j) & 1u;
  const Pow5Tables T{kPow5InvDev, kPow5Dev};
  if (FORMS && S.form && ((S.form_mask >> j) & 1u)) {
    // literal forms: how aeson prints the reference's Scientific
    const uint32_t fb = (S.form[i] >> (2 * j)) & 3u;
    if (fb & 2u) return (uint32_t)fmt_i64(S.ident[j] == 1 ? INT64_MAX : S.ident[j] == 2 ? INT64_MIN : 0, buf);
    if (fb & 1u) return (uint32_t)(f64 ? fmt_f64_integral(__builtin_bit_cast(double, v), T, buf) : fmt_i64(v, buf));
    return (uint32_t)(f64 ? fmt_f64(__builtin_bit_cast(double, v), T, buf) : fmt_i64_decimal(v, buf));
  }
  if (f64) return (uint32_t)fmt_f64(__builtin_bit_cast(double, v), T, buf, S.ident[j]);
  return (uint32_t)fmt_i64(v, buf);
}

template <bool FORMS>
__global__ __launch_bounds__(256) void k_sink_len(SinkDev S, uint64_t n, uint32_t *__restrict__ klen,
                                                  uint32_t *__restrict__ vlen) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = row_key(S, i);
    const char *p;
    uint32_t kn;
    key_text(S, k, p, kn);
    klen[i] = (S.windowed ? 16u : 0u) + frag_len(S, 0) + kn + frag_len(S, 1);
    uint32_t vn = frag_len(S, 2 + S.n_members);
    char buf[FORMS ? kNumTextIntMax : kNumTextMax];
    for (int m = 0; m < S.n_members; ++m) vn += frag_len(S, 2 + m) + member_text<FORMS>(S, m, i, k, buf, p);
    vlen[i] = vn;
  }
}

__device__ inline char *put(char *o, const char *s, uint32_t n) {
  for (uint32_t q = 0; q < n; ++q) o[q] = s[q];
  return o + n;
}

__device__ inline char *put_frag(char *o, const SinkDev &S, int f) {
  return put(o, S.frag + S.frag_off[f], frag_len(S, f));
}

template <bool FORMS>
__global__ __launch_bounds__(256) void k_sink_write(SinkDev S, uint64_t n, const uint64_t *__restrict__ koff,
                                                    const uint64_t *__restrict__ voff, char *__restrict__ kbytes,
                                                    char *__restrict__ vbytes) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t k = row_key(S, i);
    char *o = kbytes + koff[i];
    if (S.windowed) {
      // timeWindowSerde: int64BE start ++ int64BE 0
      const uint64_t w = (uint64_t)S.ws[i];
      for (int b = 0; b < 8; ++b) o[b] = (char)(w >> (56 - 8 * b));
      for (int b = 8; b < 16; ++b) o[b] = 0;
      o += 16;
    }
    const char *p;
    uint32_t kn;
    key_text(S, k, p, kn);
    o = put_frag(o, S, 0);
    o = put(o, p, kn);
    put_frag(o, S, 1);
    char *v = vbytes + voff[i];
    char buf[FORMS ? kNumTextIntMax : kNumTextMax];
    for (int m = 0; m < S.n_members; ++m) {
      v = put_frag(v, S, 2 + m);
      const uint32_t tn = member_text<FORMS>(S, m, i, k, buf, p);
      v = put(v, p, tn);
    }
    put_frag(v, S, 2 + S.n_members);
  }
}

void launch_sink_len(hipStream_t s, const SinkDev &S, uint64_t n, uint32_t *klen, uint32_t *vlen) {
  if (!n) return;
  if (S.form && S.form_mask)
    hipLaunchKernelGGL(k_sink_len<true>, dim3(grid_for(n, 256)), dim3(256), 0, s, S, n, klen, vlen);
  else
    hipLaunchKernelGGL(k_sink_len<false>, dim3(grid_for(n, 256)), dim3(256), 0, s, S, n, klen, vlen);
}

void launch_sink_write(hipStream_t s, const SinkDev &S, uint64_t n, const uint64_t *koff, const uint64_t *voff,
                       char *kbytes, char *vbytes) {
  if (!n) return;
  if (S.form && S.form_mask)
    hipLaunchKernelGGL(k_sink_write<true>, dim3(grid_for(n, 256)), dim3(256), 0, s, S, n, koff, voff, kbytes, vbytes);
  else
    hipLaunchKernelGGL(k_sink_write<false>, dim3(grid_for(n, 256)), dim3(256), 0, s, S, n, koff, voff, kbytes, vbytes);
}

}  // namespace hsg
