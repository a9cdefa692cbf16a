// Internal definitions shared by the host runtime (hsg_api.cpp) and the gfx950
// kernels (*.hip) of libhstream_gpu. Not part of the ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/hstream_gpu.h"

namespace hsg {

constexpr int kMaxCols = 8;
constexpr int kMaxAggs = 16;
constexpr int kMaxSlots = 24;   // per-group state words (8 B each)
constexpr uint64_t kEmpty = ~0ull;

// One 8-byte state word per slot; the op of each slot is fixed at op creation.
enum SlotOp : int32_t {
  S_CNT_ALL = 0,  // += 1                               (COUNT(*))
  S_CNT = 1,      // += present(col)                    (COUNT(col), AVG denominator)
  S_SUM_I = 2,    // += v (wrapping int64)              (SUM / AVG numerator of an i64 column)
  S_SUM_F = 3,    // += v (f64), identity -0.0          (SUM / AVG numerator of an f64 column)
  S_MIN_I = 4,    // min, identity INT64_MAX
  S_MAX_I = 5,    // max, identity INT64_MIN
  S_MIN_F = 6,    // min over order-preserving u64 image of the f64, identity img(2^63)
  S_MAX_F = 7,    // max over order-preserving u64 image, identity img(-2^63)
  S_LAST_SEQ = 8, // max over (global record seq + 1) of present records
  S_LAST_VAL = 9, // value of the record named by the LAST_SEQ slot just before it
  // literal forms (HSG_OPF_LITERAL_FORMS; bit 1 of a valid byte: the value's
  // JSON literal prints in Generic form, hstream_ingest.h literal_forms)
  S_CNT_DEC = 10,   // += present(col) with a decimal literal        (SUM's form)
  S_TIE_MIN = 11,   // tie word of the MIN slot slot_aux[s]: (seq + 1) << 1 | integral literal of the
                    // earliest record holding the minimum (min n x = n on ties); identity 1 (seq 0,
                    // integral: the initial maxBound wins a tie with it)
  S_TIE_MAX = 12,   // same for the MAX slot slot_aux[s], the latest record (max n x = x); identity 0
  S_LAST_FORM = 13, // max over (seq + 1) << 1 | integral literal of present records (LAST's form)
};

__host__ __device__ inline bool slot_is_form(int32_t op) { return op >= S_CNT_DEC && op <= S_LAST_FORM; }
__host__ __device__ inline bool slot_is_tie(int32_t op) { return op == S_TIE_MIN || op == S_TIE_MAX; }

// Output column j = f(slot a [, slot b]).
enum OutKind : int32_t {
  O_I64 = 0,      // slot a as int64
  O_F64 = 1,      // slot a as f64 bits
  O_F64_ORD = 2,  // slot a holds the order-preserving image of an f64
  O_AVG_I = 3,    // (double)slot a (i64 sum) / slot b (count)
  O_AVG_F = 4,    // slot a (f64 sum) / slot b (count)
};

// How output j's literal form is read (HSG_OPF_LITERAL_FORMS) from its form
// slot a (the S_CNT_DEC / S_TIE_* / S_LAST_FORM slot over the output's column)
enum FormKind : int32_t {
  F_NONE = 0,  // no form bits (COUNT, COUNT(col), AVG; ops without the flag)
  F_SUM = 1,   // a = S_CNT_DEC: integral iff 0 (a Scientific sum takes the smaller exponent)
  F_MIN = 2,   // a = S_TIE_MIN: the winning literal's bit 0; the initial value iff a == 1
  F_MAX = 3,   // a = S_TIE_MAX: the winning literal's bit 0; the initial value iff a == 0
  F_LAST = 4,  // a = S_LAST_FORM: the last present literal's bit 0; the initial value iff a == 0
};

struct Program {
  int32_t n_slots;
  int32_t n_out;
  int32_t slot_op[kMaxSlots];
  int32_t slot_col[kMaxSlots];
  int32_t out_kind[kMaxAggs];
  int32_t out_a[kMaxAggs];
  int32_t out_b[kMaxAggs];
  int32_t form_kind[kMaxAggs];  // FormKind
  int32_t form_a[kMaxAggs];
  int32_t slot_aux[kMaxSlots];  // S_TIE_*: the MIN / MAX slot the tie word belongs to
  int32_t ties;                 // the program has S_TIE_* slots
  // per-record changelog of one-window ops (k_pr_bucket -> k_pr_emit1): each
  // record's state as the outputs read it -- fin_n slots (fin_slot) and, with
  // fin_form, the row's literal-form word -- when that is fewer words than
  // the state (LAST's sequence, tie words, decimal counts stay behind)
  int32_t fin_n;
  int32_t fin_form;
  int32_t fin_slot[kMaxSlots];
};
// words per record of that projection
__host__ __device__ inline int prog_fin_words(const Program &p) { return p.fin_n + p.fin_form; }

// u64 division by an invariant divisor (Granlund–Montgomery), exact for all n.
struct Divider {
  uint64_t d;
  uint64_t m;
  int32_t sh1;
  int32_t sh2;
};

__host__ __device__ inline uint64_t umulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ inline uint64_t udiv(const Divider &v, uint64_t n) {
  uint64_t t = umulhi64(v.m, n);
  return (t + ((n - t) >> v.sh1)) >> v.sh2;
}

inline Divider make_divider(uint64_t d) {
  Divider v;
  v.d = d;
  int l = 0;
  while (l < 64 && (1ull << l) < d) ++l;  // l = ceil(log2 d)
  unsigned __int128 two_l = (unsigned __int128)1 << l;
  unsigned __int128 m = (((unsigned __int128)1 << 64) * (two_l - d)) / d + 1;
  v.m = (uint64_t)m;
  v.sh1 = l < 1 ? l : 1;
  v.sh2 = l - 1 > 0 ? l - 1 : 0;
  return v;
}

// Device-side per-op scalars (one 512-byte block, zeroed / set per batch).
struct DevScalars {
  int64_t wm_out;        // watermark after the batch
  int64_t k_epoch;       // window index represented by k_rel = 0
  uint32_t epoch_set;
  uint32_t err;          // bit0 OOM, bit1 RANGE
  uint64_t pairs;        // accepted (record, window) updates
  uint64_t late;         // rejected by grace
  uint64_t out_rows;     // rows appended to the changelog this batch
  uint64_t touched;
  uint64_t live;         // dump: rows found
  uint32_t no_late;      // this batch: no (record, window) can fail the grace check
  uint32_t redo;         // optimistic partition path: the batch has late records, run it again carefully
  uint64_t packed;       // partition path, this batch: records in the packed layout (hsg_part.h)
  uint64_t kbase;        // packed layout: window (relative to the epoch) the 16-bit window offsets count from
  uint64_t scratch[45];  // [0] groups flushed (partition path), [1] touched-list length, [8..20] phase clocks,
                         // [21..22] optimistic pass ts extrema, [31] lean partials of the batch (bound on
                         // its new groups), [32] held back for table room: bit 0 lean apply, bit 1 general,
                         // bit 2 k_seg_apply, [33] groups claimed in the table's overflow rows (TwTable::ovf),
                         // [34] k_seg_apply's deferred window updates (bound on their new groups)
  uint64_t live_x[8];    // more rows found, one shard per XCD (blockIdx & 7) for kernels whose every
                         // workgroup adds; the host folds them into `live` when it fetches the scalars
};
constexpr int kScratchWords = 45;
static_assert(sizeof(DevScalars) == 512, "DevScalars layout");

constexpr uint32_t ERR_OOM = 1u;
constexpr uint32_t ERR_RANGE = 2u;

// Changelog / dump rows in HBM, columnar.
struct OutCols {
  uint32_t *key;
  int64_t *ws;
  int64_t *we;
  int64_t *src;
  int64_t *agg[kMaxAggs];  // 8-byte words (i64 or f64 bits)
  uint32_t *form;          // literal forms (hsg_rows.form), null = not kept
};

struct Batch {
  uint64_t n;
  const uint32_t *key;
  const int64_t *ts;
  const int64_t *col[kMaxCols];  // i64 or f64 bits
  const uint8_t *valid[kMaxCols];
};

// Time-window (tumbling / hopping / unwindowed) hash state in HBM, one row per
// (key, window) group, array-of-structs so a group is one cache line:
//   word 0      group key = key_id << 32 | (k - k_epoch); kEmpty = free
//   word 1      low 32 bits: id of the last batch that touched the group
//   words 2..   aggregate slots (n_slots words)
// Rows are `stride` words (a power of two up to 16, so a row never straddles a
// 128-byte line). The home slot keeps the 8 windows of an aligned window block
// of one key in 8 consecutive rows (see tw_home).
struct TwTable {
  uint64_t *rows;   // [cap + overflow][stride]
  uint64_t mask;    // cap - 1 (the region slots)
  uint32_t stride;  // words per row
  uint32_t blocked; // window-block home slots, probe step 8 (windowed ops with >= 8 slots)
  uint64_t rmask;   // slots per region - 1 (regions = 2^rbits, see hsg_tw.h)
  int32_t rbits;    // region bits of the key hash (below the owner bits)
  int32_t bshift;   // owner bits of the key hash (multi-GPU)
  uint8_t *dirty;   // [slots() / 8]: 8-slot blocks claimed since the last clear (null: not kept)
  uint64_t omask;   // overflow slots - 1: rows [cap, cap + omask + 1) take the groups whose
                    // region probe found no free slot (hsg_tw.h tw_ovf_claim)
  uint64_t *ovf;    // device counter of overflow claims (DevScalars scratch[33]: per batch)
  __host__ __device__ uint64_t slots() const { return mask + 1 + omask + 1; }
  __host__ __device__ uint64_t *key(uint64_t s) const { return rows + s * stride; }
  // every claim marks its block, so a clear rewrites only the claimed blocks
  __device__ void mark(uint64_t s) const {
    if (dirty) dirty[s >> 3] = 1;
  }
  __host__ __device__ uint32_t *stamp(uint64_t s) const { return (uint32_t *)(rows + s * stride + 1); }
  __host__ __device__ int64_t *aggs(uint64_t s) const { return (int64_t *)(rows + s * stride + 2); }
};

// overflow rows after a table of `cap` region slots: 1/8 of it (>= 64)
inline uint64_t tw_ovf_slots(uint64_t cap) { return cap / 8 > 64 ? cap / 8 : 64; }

inline uint32_t tw_row_stride(int n_slots) {
  uint32_t w = 2u + (uint32_t)n_slots, s = 4;
  while (s < w && s < 16) s <<= 1;
  return s >= w ? s : (w + 7u) & ~7u;
}

struct TwParams {
  int32_t kind;     // hsg_window_kind
  int32_t batch_id;
  int64_t size;
  int64_t adv;
  int64_t grace;
  int64_t wm_in;
  uint64_t rec_base; // global seq of record 0 of this batch
  Divider div;
};

__device__ __host__ inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  x ^= x >> 33;
  return x;
}

// Hash of a group key: its top bits pick the owner GPU (power-of-two ranks),
// the next bits the partition bucket, the bits below the aggregation round.
// Key hash whose TOP bits pick the owner GPU, the partition bucket, the table
// region and the key-hash rounds (every user takes bits from the top, at most
// 32 of them): a 32-bit finaliser (murmur3 fmix32) in the high word -- 32-bit
// multiplies only, it runs for every record in the histogram and scatter
// passes -- and a cheaper second mix in the low word.
__device__ __host__ inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}
__device__ __host__ inline uint64_t key_hash(uint32_t key) {
  const uint32_t h = fmix32(key * 0x9E3779B1u + 0x632BE59Bu);
  return ((uint64_t)h << 32) | (uint32_t)((h * 0x27D4EB2Fu) ^ key);
}
__device__ __host__ inline int log2_exact(uint32_t g) {  // -1 unless g is a power of two
  if (g == 0 || (g & (g - 1))) return -1;
  int l = 0;
  while ((1u << l) < g) ++l;
  return l;
}

// Order-preserving map f64 -> u64 (total order on non-NaN values).
__device__ __host__ inline uint64_t f64_ord(double d) {
  uint64_t u = __builtin_bit_cast(uint64_t, d);
  return (u & 0x8000000000000000ull) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __host__ inline double f64_unord(uint64_t o) {
  uint64_t u = (o & 0x8000000000000000ull) ? (o & 0x7fffffffffffffffull) : ~o;
  return __builtin_bit_cast(double, u);
}

inline int64_t slot_identity(int32_t op) {
  switch (op) {
    case S_MIN_I: return INT64_MAX;
    case S_MAX_I: return INT64_MIN;
    case S_MIN_F: return (int64_t)f64_ord((double)INT64_MAX);
    case S_MAX_F: return (int64_t)f64_ord((double)INT64_MIN);
    case S_SUM_F: return INT64_MIN;  // -0.0: x + -0.0 == x for every x, and a SUM nothing reached stays -0.0
    case S_TIE_MIN: return 1;
    default: return 0;
  }
}
// the op keeps literal forms (its slots read bit 1 of the valid bytes, which
// only the generic record paths carry: not the partition layouts)
inline bool prog_has_forms(const Program &p) {
  for (int s = 0; s < p.n_slots; ++s)
    if (slot_is_form(p.slot_op[s])) return true;
  return false;
}
// the op's slots need each record's global sequence number
inline bool prog_needs_seq(const Program &p) {
  for (int s = 0; s < p.n_slots; ++s)
    if (p.slot_op[s] == S_LAST_SEQ || slot_is_tie(p.slot_op[s]) || p.slot_op[s] == S_LAST_FORM) return true;
  return false;
}
// the partitioned records carry the sequence word (hsg_dev.h seq_word: global
// seq + 1 and the decimal-literal bits) for these ops
inline bool prog_part_seq(const Program &p) { return prog_needs_seq(p) || prog_has_forms(p); }
inline bool prog_has_tie(const Program &p) {
  for (int s = 0; s < p.n_slots; ++s)
    if (slot_is_tie(p.slot_op[s])) return true;
  return false;
}

// ---- kernel launchers (defined in the .hip files) --------------------------
struct RowPtrs {
  int64_t *p[kMaxAggs];
};
void launch_clear_scalars(hipStream_t s, DevScalars *sc);
// copy into the pinned host mirror h, then clear (the end of a push)
void launch_fetch_clear_scalars(hipStream_t s, DevScalars *sc, DevScalars *h);
void launch_copy_rows(hipStream_t s, const OutCols &src, uint64_t from, uint64_t n, int n_aggs, uint32_t *key,
                      int64_t *ws, int64_t *we, int64_t *si, const RowPtrs &aggs, uint32_t *form = nullptr);
void launch_fill_u64(hipStream_t s, uint64_t *p, uint64_t n, uint64_t v);
void launch_fill_rows(hipStream_t s, int64_t *aggs, uint64_t rows, const Program &prog);
// every row of a time-window table: key EMPTY, stamp 0, aggregate identities
// whole table (and its dirty map, when kept)
void launch_tw_reset(hipStream_t s, const TwTable &t, const Program &prog);
// only the blocks the dirty map marks (the map must cover every claim since
// the last launch_tw_reset); *cnt (device) <- the dirty blocks counted
void launch_tw_reset_dirty(hipStream_t s, const TwTable &t, const Program &prog, uint64_t *cnt);
// one byte per 8-slot block, padded to 16 bytes
inline uint64_t tw_dirty_bytes(uint64_t cap) { return ((cap >> 3) + 16) & ~15ull; }
void launch_fill_u32(hipStream_t s, uint32_t *p, uint64_t n, uint32_t v);

// narrow transport columns of a batch (include/hstream_gpu.h hsg_enc) into
// the op's full-width staging, on the device after the H2D
struct WidenArgs {
  uint64_t n;
  const uint16_t *k16;           // null: key_id is not narrow
  uint32_t *key;
  const int32_t *ts32;           // null: ts is not TS32
  int64_t ts_base;
  const uint16_t *ts16;          // null: ts is not TS16
  const int64_t *frames;         // TS16: a base per HSG_TS16_FRAME records
  int64_t *ts;
  const int32_t *c32[kMaxCols];  // null: the column is not narrow
  int64_t *col[kMaxCols];        // int64 words (i64 or f64 bits)
  double div[kMaxCols];          // HSG_ENC_DEC32: 10^scale; 0: HSG_ENC_I32
};
void launch_widen(hipStream_t s, const WidenArgs &w);
// dump ordering on the device (op_device.cpp sort_dump_rows_device): the
// window index of each row (ws / adv - k_epoch) and the identity permutation;
// then one 4-/8-byte column gathered through a permutation
void launch_dump_keys(hipStream_t s, const int64_t *ws, uint64_t n, int64_t adv, int64_t k_epoch, uint32_t *k, uint32_t *v);
void launch_gather_u32(hipStream_t s, const uint32_t *src, const uint32_t *perm, uint64_t n, uint32_t *dst);
void launch_gather_u64(hipStream_t s, const uint64_t *src, const uint32_t *perm, uint64_t n, uint64_t *dst);
inline bool batch_narrow(const hsg_batch *b) {
  bool any = b->ts_enc != HSG_ENC_FULL || b->key_enc != HSG_ENC_FULL;
  for (int c = 0; c < b->n_cols && c < kMaxCols; ++c) any |= b->col_enc[c] != HSG_ENC_FULL;
  return any;
}

// stream time: tile maxima -> exclusive tile prefix (+ epoch init)
void launch_tile_stats(hipStream_t s, const Batch &b, int64_t *tile_max, int64_t *tile_min, uint64_t n_tiles);
// grace >= 0: also decide sc->no_late for a time-window op
// window epoch from the first keyed record (ts >= 0) of the batch, when not
// yet set: optimistic batches need no stream-time pass for it
void launch_epoch_first(hipStream_t s, const Batch &b, int64_t adv, DevScalars *sc);
void launch_tile_scan(hipStream_t s, const int64_t *tile_max, const int64_t *tile_min, int64_t *tile_prefix,
                      uint64_t n_tiles, int64_t wm_in, int64_t adv, bool set_epoch, DevScalars *sc,
                      int64_t grace = -1);

// time windows, atomic hash aggregation (per-batch / none modes). rec_wm / seq
// (optional) carry per-record stream time and global sequence after a key
// exchange; last_pass = the LAST-value resolution pass.
void launch_tw_agg(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const Program &prog,
                   const int64_t *tile_prefix, const int64_t *rec_wm, const int64_t *seq, DevScalars *sc,
                   bool last_pass);
// emit rows whose stamp == batch_id (mode 0) or every live row (mode 1) in slot
// order; *total (device) receives the row count
constexpr uint64_t kEmitChunk = 4096;
struct EmitScratch {
  uint32_t *cnt;     // [emit_chunks(cap)]
  uint64_t *off;     // [emit_chunks(cap)]
  uint64_t *partial; // scan partials
};
uint64_t emit_chunks(uint64_t cap);
void launch_tw_emit(hipStream_t s, const TwTable &t, uint64_t cap, const Program &prog, const TwParams &p, int mode,
                    OutCols out, uint64_t out_base, uint64_t out_cap, DevScalars *sc, const EmitScratch &es,
                    uint64_t *total);
// retention (retention.cpp): rows closed at p.wm_in (end + grace <= stream
// time). dst == nullptr: count them (*total, device; es.off = chunk offsets);
// else copy them, raw row words in slot order, to dst (after the count).
void launch_tw_closed(hipStream_t s, const TwTable &t, uint64_t cap, const TwParams &p, const DevScalars *sc,
                      const EmitScratch &es, uint64_t *total, uint64_t *dst);
// rows src[0, n) (stride = dst.stride words) into dst, skipping empty rows
// and, with skip_closed, closed ones; *kept += rows inserted
void launch_tw_reinsert(hipStream_t s, const uint64_t *src, uint64_t n, const TwTable &dst, const TwParams &p,
                        DevScalars *sc, bool skip_closed, unsigned long long *kept);
unsigned grid_for(uint64_t n, unsigned tpb);
// touched list (hsg_part.h) across a table rebuild: slots -> group keys in the
// old table, group keys -> slots in the new one (kTouchSkipEntry kept)
constexpr uint32_t kTouchSkipEntry = 0xFFFFFFFFu;
void launch_touch_keys(hipStream_t s, const TwTable &t, const uint32_t *touched, uint64_t n, uint64_t *keys);
void launch_touch_slots(hipStream_t s, const TwTable &t, const uint64_t *keys, uint64_t n, uint32_t *touched);

constexpr int kTileThreads = 256;
constexpr int kRecPerThread = 4;
constexpr int kTileRecords = kTileThreads * kRecPerThread;

}  // namespace hsg
