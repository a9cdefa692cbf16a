// Host orchestration of the stream-stream join (include/hstream_join.h,
// hsg_join.h): per batch, the LSD sort of the records by (record key, side,
// ts) and by (side, ts), rank merges with the resident state and timestamp
// set, the probe (count, scan, write), and the compactions that form the
// next state. Every launch is on the join's own stream.
#include <hip/hip_runtime.h>

#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/hstream_join.h"
#include "hsg_exchange.h"
#include "hsg_join.h"
#include "hsg_sort.h"

using namespace hsg;

namespace hsg {
// hsg_api.cpp
int engine_device(const hsg_engine *e);
// a communicator of the engine's ranks for one sharded object (nullptr, rank
// 0 of 1 on a single-rank engine)
int engine_split_comm(hsg_engine *e, Comm **out, int *rank, int *nranks, std::string &err);
}

struct hsg_join {
  int device = 0;
  hipStream_t stream = nullptr;
  int64_t before = 0, after = 0;
  uint64_t batch_cap = 0;
  std::string err;
  // batch scratch (batch_cap)
  uint8_t *st_side = nullptr;
  uint32_t *st_key = nullptr, *st_jkey = nullptr;
  int64_t *st_ts = nullptr;
  uint64_t *st_handle = nullptr;
  JEnt *braw = nullptr, *bs = nullptr, *bt = nullptr;
  uint32_t *perm0 = nullptr, *perm1 = nullptr, *key0 = nullptr, *key1 = nullptr, *pos = nullptr, *cnt = nullptr;
  uint64_t *off = nullptr;
  TEnt *tb = nullptr;
  void *sort_scratch = nullptr;
  // state
  JEnt *R = nullptr, *Rn = nullptr, *M = nullptr;
  uint64_t nR = 0, r_cap = 0;
  TEnt *T = nullptr, *Tn = nullptr, *Tm = nullptr;
  uint64_t nT = 0, t_cap = 0;
  // state-sized scratch
  uint32_t *flag = nullptr;
  uint64_t *soff = nullptr, *partial = nullptr, *tot = nullptr;
  uint64_t s_cap = 0;
  uint64_t *h_tot = nullptr;  // pinned [4]
  // output rows
  JoinOut out = {};
  uint64_t out_cap = 0, pending = 0;
  // sharded (the engine's ranks > 1): each rank pushes its slice of the
  // poll batch; the slices are all-gathered into the global batch (rank
  // order = arrival order), every rank keeps the whole timestamp set (the
  // end-point rule reads any key's entries) and stores / probes the records
  // whose key it owns (join_owner), so its rows are those records' rows
  Comm *comm = nullptr;
  int rank = 0, nranks = 1;
  int64_t *d_n = nullptr, *d_nall = nullptr, *h_nall = nullptr;  // slice sizes (device, all-gathered, pinned)
  int64_t *d_off = nullptr;                                       // [G + 1] slice offsets
  uint8_t *r_side = nullptr;                                      // [G * batch_cap] all-gathered slots
  uint32_t *r_key = nullptr, *r_jkey = nullptr;
  int64_t *r_ts = nullptr;
  uint64_t *r_handle = nullptr;
  uint8_t *g_side = nullptr;                                      // [G * batch_cap] the global batch
  uint32_t *g_key = nullptr, *g_jkey = nullptr;
  int64_t *g_ts = nullptr;
  uint64_t *g_handle = nullptr;
};

namespace {

#define JTRY(expr)                                                          \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) {                                                 \
      j->err = std::string(#expr) + ": " + hipGetErrorString(_e);           \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;          \
    }                                                                       \
  } while (0)

template <typename T>
hipError_t dmalloc(T *&p, uint64_t count) {
  return hipMalloc((void **)&p, (count ? count : 1) * sizeof(T));
}

void dfree(void *p) {
  if (p) hipFree(p);
}

void free_join(hsg_join *j) {
  if (!j) return;
  hipSetDevice(j->device);
  if (j->stream) hipStreamSynchronize(j->stream);
  void *ptrs[] = {j->st_side, j->st_key, j->st_jkey, j->st_ts, j->st_handle, j->braw, j->bs, j->bt, j->perm0,
                  j->perm1, j->key0, j->key1, j->pos, j->cnt, j->off, j->tb, j->sort_scratch, j->R, j->Rn, j->M,
                  j->T, j->Tn, j->Tm, j->flag, j->soff, j->partial, j->tot, j->out.this_h, j->out.other_h,
                  j->out.jkey, j->out.ts};
  for (void *p : ptrs) dfree(p);
  void *xptrs[] = {j->d_n, j->d_nall, j->d_off, j->r_side, j->r_key, j->r_jkey, j->r_ts, j->r_handle,
                   j->g_side, j->g_key, j->g_jkey, j->g_ts, j->g_handle};
  for (void *p : xptrs) dfree(p);
  if (j->h_nall) hipHostFree(j->h_nall);
  if (j->comm) comm_destroy(j->comm);
  if (j->h_tot) hipHostFree(j->h_tot);
  if (j->stream) hipStreamDestroy(j->stream);
  delete j;
}

// state arrays with room for `need` entries (contents of R / T kept)
int ensure_state(hsg_join *j, uint64_t r_need, uint64_t t_need) {
  if (r_need > j->r_cap) {
    uint64_t c = j->r_cap ? j->r_cap : (1u << 16);
    while (c < r_need) c *= 2;
    JEnt *R = nullptr, *Rn = nullptr, *M = nullptr;
    JTRY(dmalloc(R, c));
    JTRY(dmalloc(Rn, c));
    JTRY(dmalloc(M, c));
    if (j->nR) JTRY(hipMemcpyAsync(R, j->R, j->nR * sizeof(JEnt), hipMemcpyDeviceToDevice, j->stream));
    JTRY(hipStreamSynchronize(j->stream));
    dfree(j->R);
    dfree(j->Rn);
    dfree(j->M);
    j->R = R, j->Rn = Rn, j->M = M, j->r_cap = c;
  }
  if (t_need > j->t_cap) {
    uint64_t c = j->t_cap ? j->t_cap : (1u << 16);
    while (c < t_need) c *= 2;
    TEnt *T = nullptr, *Tn = nullptr, *Tm = nullptr;
    JTRY(dmalloc(T, c));
    JTRY(dmalloc(Tn, c));
    JTRY(dmalloc(Tm, c));
    if (j->nT) JTRY(hipMemcpyAsync(T, j->T, j->nT * sizeof(TEnt), hipMemcpyDeviceToDevice, j->stream));
    JTRY(hipStreamSynchronize(j->stream));
    dfree(j->T);
    dfree(j->Tn);
    dfree(j->Tm);
    j->T = T, j->Tn = Tn, j->Tm = Tm, j->t_cap = c;
  }
  // flags / offsets of the state compaction (M) and the timestamp set (Tm) side by side
  const uint64_t s_need = j->r_cap + j->t_cap + 2;
  if (s_need > j->s_cap) {
    dfree(j->flag);
    dfree(j->soff);
    dfree(j->partial);
    j->flag = nullptr, j->soff = nullptr, j->partial = nullptr;
    JTRY(dmalloc(j->flag, s_need));
    JTRY(dmalloc(j->soff, s_need + 1));
    JTRY(dmalloc(j->partial, scan_partials_needed(s_need) + 8));
    j->s_cap = s_need;
  }
  return HSG_OK;
}

int ensure_out(hsg_join *j, uint64_t need) {
  if (need <= j->out_cap) return HSG_OK;
  uint64_t c = j->out_cap ? j->out_cap : (1u << 16);
  while (c < need) c *= 2;
  JoinOut o = {};
  JTRY(dmalloc(o.this_h, c));
  JTRY(dmalloc(o.other_h, c));
  JTRY(dmalloc(o.jkey, c));
  JTRY(dmalloc(o.ts, c));
  if (j->pending) {
    const hipMemcpyKind k = hipMemcpyDeviceToDevice;
    JTRY(hipMemcpyAsync(o.this_h, j->out.this_h, j->pending * 8, k, j->stream));
    JTRY(hipMemcpyAsync(o.other_h, j->out.other_h, j->pending * 8, k, j->stream));
    JTRY(hipMemcpyAsync(o.jkey, j->out.jkey, j->pending * 4, k, j->stream));
    JTRY(hipMemcpyAsync(o.ts, j->out.ts, j->pending * 8, k, j->stream));
  }
  JTRY(hipStreamSynchronize(j->stream));
  dfree(j->out.this_h);
  dfree(j->out.other_h);
  dfree(j->out.jkey);
  dfree(j->out.ts);
  j->out = o;
  j->out_cap = c;
  return HSG_OK;
}

// stable LSD sort of the batch entries' indices over the given passes
uint32_t *sort_perm(hsg_join *j, uint64_t n, const int *passes, int np) {
  static const int bits[4] = {32, 32, 2, 32};
  launch_join_iota(j->stream, j->perm0, n);
  uint32_t *p = j->perm0, *q = j->perm1;
  for (int i = 0; i < np; ++i) {
    launch_join_sortkey(j->stream, j->braw, p, n, passes[i], j->key0);
    const int which = radix_sort_pairs(j->stream, j->key0, p, j->key1, q, n, bits[passes[i]], j->sort_scratch);
    if (which) {
      uint32_t *t = p;
      p = q;
      q = t;
    }
  }
  return p;
}

}  // namespace

extern "C" int hsg_join_create(hsg_engine *eng, const hsg_join_config *cfg, hsg_join **out) {
  if (!eng || !cfg || !out || cfg->before_ms < 0 || cfg->after_ms < 0 || cfg->batch_capacity == 0 ||
      cfg->batch_capacity >= 0x7FFFFFFFull)
    return HSG_E_INVALID;
  *out = nullptr;
  hsg_join *j = new (std::nothrow) hsg_join();
  if (!j) return HSG_E_OOM;
  j->device = engine_device(eng);
  j->before = cfg->before_ms;
  j->after = cfg->after_ms;
  j->batch_cap = cfg->batch_capacity;
  {
    std::string err;
    const int rc = engine_split_comm(eng, &j->comm, &j->rank, &j->nranks, err);
    if (rc != HSG_OK) {
      free_join(j);
      return rc;
    }
  }
  const int G = j->nranks;
  // (sharded: the global batch holds every rank's slice)
  const uint64_t n = j->batch_cap * (uint64_t)G;
  hipError_t e = hipSetDevice(j->device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&j->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = dmalloc(j->st_side, n);
  if (e == hipSuccess) e = dmalloc(j->st_key, n);
  if (e == hipSuccess) e = dmalloc(j->st_jkey, n);
  if (e == hipSuccess) e = dmalloc(j->st_ts, n);
  if (e == hipSuccess) e = dmalloc(j->st_handle, n);
  if (e == hipSuccess) e = dmalloc(j->braw, n);
  if (e == hipSuccess) e = dmalloc(j->bs, n);
  if (e == hipSuccess) e = dmalloc(j->bt, n);
  if (e == hipSuccess) e = dmalloc(j->perm0, n);
  if (e == hipSuccess) e = dmalloc(j->perm1, n);
  if (e == hipSuccess) e = dmalloc(j->key0, n);
  if (e == hipSuccess) e = dmalloc(j->key1, n);
  if (e == hipSuccess) e = dmalloc(j->pos, n);
  if (e == hipSuccess) e = dmalloc(j->cnt, n);
  if (e == hipSuccess) e = dmalloc(j->off, n + 1);
  if (e == hipSuccess) e = dmalloc(j->tb, n);
  if (e == hipSuccess) e = hipMalloc(&j->sort_scratch, sort_scratch_bytes(n));
  if (e == hipSuccess) e = dmalloc(j->tot, 4);
  if (e == hipSuccess) e = hipHostMalloc((void **)&j->h_tot, 4 * sizeof(uint64_t), hipHostMallocDefault);
  if (G > 1) {
    if (e == hipSuccess) e = dmalloc(j->d_n, 1);
    if (e == hipSuccess) e = dmalloc(j->d_nall, G);
    if (e == hipSuccess) e = dmalloc(j->d_off, G + 1);
    if (e == hipSuccess) e = hipHostMalloc((void **)&j->h_nall, (G + 1) * sizeof(int64_t), hipHostMallocDefault);
    if (e == hipSuccess) e = dmalloc(j->r_side, n);
    if (e == hipSuccess) e = dmalloc(j->r_key, n);
    if (e == hipSuccess) e = dmalloc(j->r_jkey, n);
    if (e == hipSuccess) e = dmalloc(j->r_ts, n);
    if (e == hipSuccess) e = dmalloc(j->r_handle, n);
    if (e == hipSuccess) e = dmalloc(j->g_side, n);
    if (e == hipSuccess) e = dmalloc(j->g_key, n);
    if (e == hipSuccess) e = dmalloc(j->g_jkey, n);
    if (e == hipSuccess) e = dmalloc(j->g_ts, n);
    if (e == hipSuccess) e = dmalloc(j->g_handle, n);
  }
  if (e != hipSuccess) {
    free_join(j);
    return e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;
  }
  int rc = ensure_state(j, n, n);
  if (rc == HSG_OK) rc = ensure_out(j, n);
  if (rc != HSG_OK) {
    free_join(j);
    return rc;
  }
  *out = j;
  return HSG_OK;
}

extern "C" void hsg_join_destroy(hsg_join *j) { free_join(j); }

extern "C" const char *hsg_join_last_error(const hsg_join *j) { return j ? j->err.c_str() : "null join"; }

extern "C" int hsg_join_push(hsg_join *j, const hsg_join_batch *b) {
  if (!j || !b) return HSG_E_INVALID;
  if (b->n > j->batch_cap) {
    j->err = "batch larger than batch_capacity";
    return HSG_E_CAPACITY;
  }
  if (b->mem != HSG_MEM_HOST && b->mem != HSG_MEM_DEVICE) return HSG_E_INVALID;
  uint64_t n = b->n;
  if (n && (!b->side || !b->key_id || !b->join_key || !b->ts || !b->handle)) return HSG_E_INVALID;
  if (!n && j->nranks == 1) return HSG_OK;  // (sharded: every rank joins the all-gather, empty slice or not)
  try {
    JTRY(hipSetDevice(j->device));
    hipStream_t s = j->stream;
    JoinBatchDev db;
    db.n = n;
    db.rank = (uint32_t)j->rank;
    db.nranks = (uint32_t)j->nranks;
    if (b->mem == HSG_MEM_DEVICE && j->nranks == 1) {
      db.side = b->side, db.key = b->key_id, db.jkey = b->join_key, db.ts = b->ts, db.handle = b->handle;
    } else if (n) {
      const hipMemcpyKind k = b->mem == HSG_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
      JTRY(hipMemcpyAsync(j->st_side, b->side, n, k, s));
      JTRY(hipMemcpyAsync(j->st_key, b->key_id, n * 4, k, s));
      JTRY(hipMemcpyAsync(j->st_jkey, b->join_key, n * 4, k, s));
      JTRY(hipMemcpyAsync(j->st_ts, b->ts, n * 8, k, s));
      JTRY(hipMemcpyAsync(j->st_handle, b->handle, n * 8, k, s));
      db.side = j->st_side, db.key = j->st_key, db.jkey = j->st_jkey, db.ts = j->st_ts, db.handle = j->st_handle;
    }
    if (j->nranks > 1) {
      // every rank's slice size, then the slices (padded to the largest) and
      // the global batch in rank order
      const int G = j->nranks;
      j->h_nall[0] = (int64_t)n;
      JTRY(hipMemcpyAsync(j->d_n, j->h_nall, 8, hipMemcpyHostToDevice, s));
      int rc = comm_allgather(j->comm, j->d_n, j->d_nall, 1, ncclInt64, 8, s, j->err);
      if (rc != HSG_OK) return rc;
      JTRY(hipMemcpyAsync(j->h_nall, j->d_nall, G * 8, hipMemcpyDeviceToHost, s));
      JTRY(hipStreamSynchronize(s));
      uint64_t mx = 0, tot = 0;
      std::vector<int64_t> off(G + 1, 0);
      for (int q = 0; q < G; ++q) {
        const uint64_t nq = (uint64_t)j->h_nall[q];
        mx = nq > mx ? nq : mx;
        off[q] = (int64_t)tot;
        tot += nq;
      }
      off[G] = (int64_t)tot;
      if (!tot) return HSG_OK;  // (every rank saw the same sizes)
      if (mx > j->batch_cap) {
        j->err = "a rank's batch is larger than batch_capacity";
        return HSG_E_CAPACITY;
      }
      JTRY(hipMemcpyAsync(j->d_off, off.data(), (G + 1) * 8, hipMemcpyHostToDevice, s));
      JTRY(hipStreamSynchronize(s));  // (off is a host temporary)
      if ((rc = comm_group_start(j->comm, j->err)) != HSG_OK) return rc;
      if ((rc = comm_allgather(j->comm, j->st_side, j->r_side, mx, ncclUint8, 1, s, j->err)) != HSG_OK) return rc;
      if ((rc = comm_allgather(j->comm, j->st_key, j->r_key, mx, ncclUint32, 4, s, j->err)) != HSG_OK) return rc;
      if ((rc = comm_allgather(j->comm, j->st_jkey, j->r_jkey, mx, ncclUint32, 4, s, j->err)) != HSG_OK) return rc;
      if ((rc = comm_allgather(j->comm, j->st_ts, j->r_ts, mx, ncclInt64, 8, s, j->err)) != HSG_OK) return rc;
      if ((rc = comm_allgather(j->comm, j->st_handle, j->r_handle, mx, ncclUint64, 8, s, j->err)) != HSG_OK)
        return rc;
      if ((rc = comm_group_end(j->comm, j->err)) != HSG_OK) return rc;
      JoinBatchDev slots = db;
      slots.side = j->r_side, slots.key = j->r_key, slots.jkey = j->r_jkey, slots.ts = j->r_ts,
      slots.handle = j->r_handle;
      launch_join_compact(s, slots, mx, j->d_off, G, tot, j->g_side, j->g_key, j->g_jkey, j->g_ts, j->g_handle);
      n = tot;
      db.n = n;
      db.side = j->g_side, db.key = j->g_key, db.jkey = j->g_jkey, db.ts = j->g_ts, db.handle = j->g_handle;
    }
    int rc = ensure_state(j, j->nR + n, j->nT + n);
    if (rc != HSG_OK) return rc;
    launch_join_build(s, db, j->braw);
    // 1. the batch by (record key, side, ts, arrival), merged into the state
    static const int m_passes[4] = {0, 1, 2, 3};
    uint32_t *perm = sort_perm(j, n, m_passes, 4);
    launch_join_gather(s, j->braw, perm, n, j->bs);
    launch_join_merge(s, j->R, j->nR, j->bs, n, j->M, j->pos);
    const uint64_t nM = j->nR + n;
    // 2. the batch's timestamps by (side, ts, arrival), merged into the set
    static const int t_passes[3] = {0, 1, 2};
    perm = sort_perm(j, n, t_passes, 3);
    launch_join_gather(s, j->braw, perm, n, j->bt);
    launch_join_tflags(s, j->bt, n, j->flag);
    scan_excl_u32(s, j->flag, j->soff, n, j->partial, j->tot);
    launch_join_twrite(s, j->bt, n, j->flag, j->soff, j->tb);
    JTRY(hipMemcpyAsync(j->h_tot, j->tot, 8, hipMemcpyDeviceToHost, s));
    JTRY(hipStreamSynchronize(s));
    const uint64_t ntb = j->h_tot[0];
    launch_join_tmerge(s, j->T, j->nT, j->tb, ntb, j->Tm);
    const uint64_t nTm = j->nT + ntb;
    // 3. probe: counts, offsets, rows
    JoinOut none = {};
    launch_join_probe(s, j->M, nM, j->pos, n, j->Tm, nTm, j->before, j->after, j->cnt, nullptr, none, 0);
    scan_excl_u32(s, j->cnt, j->off, n, j->partial, j->tot + 1);
    JTRY(hipMemcpyAsync(j->h_tot + 1, j->tot + 1, 8, hipMemcpyDeviceToHost, s));
    JTRY(hipStreamSynchronize(s));
    const uint64_t rows = j->h_tot[1];
    rc = ensure_out(j, j->pending + rows);
    if (rc != HSG_OK) return rc;
    if (rows)
      launch_join_probe(s, j->M, nM, j->pos, n, j->Tm, nTm, j->before, j->after, j->cnt, j->off, j->out, j->pending);
    // 4. next state and timestamp set
    launch_join_rflags(s, j->M, nM, j->flag);
    scan_excl_u32(s, j->flag, j->soff, nM, j->partial, j->tot + 2);
    launch_join_rwrite(s, j->M, nM, j->flag, j->soff, j->Rn);
    launch_join_tkeep(s, j->Tm, nTm, j->flag + nM);
    scan_excl_u32(s, j->flag + nM, j->soff + nM + 1, nTm, j->partial, j->tot + 3);
    launch_join_tkeep_write(s, j->Tm, nTm, j->flag + nM, j->soff + nM + 1, j->Tn);
    JTRY(hipMemcpyAsync(j->h_tot + 2, j->tot + 2, 16, hipMemcpyDeviceToHost, s));
    JTRY(hipStreamSynchronize(s));
    JTRY(hipGetLastError());
    JEnt *t = j->R;
    j->R = j->Rn, j->Rn = t;
    TEnt *u = j->T;
    j->T = j->Tn, j->Tn = u;
    j->nR = j->h_tot[2];
    j->nT = j->h_tot[3];
    j->pending += rows;
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  }
}

extern "C" int hsg_join_pending(const hsg_join *j, uint64_t *n) {
  if (!j || !n) return HSG_E_INVALID;
  *n = j->pending;
  return HSG_OK;
}

extern "C" int hsg_join_state_rows(const hsg_join *j, uint64_t *n) {
  if (!j || !n) return HSG_E_INVALID;
  *n = j->nR;
  return HSG_OK;
}

extern "C" int hsg_join_drain(hsg_join *jj, hsg_join_rows *o, uint64_t *n_out) {
  hsg_join *j = jj;
  if (!j || !o || !n_out) return HSG_E_INVALID;
  *n_out = j->pending;
  if (o->capacity < j->pending) return HSG_E_CAPACITY;
  if (o->mem != HSG_MEM_HOST && o->mem != HSG_MEM_DEVICE) return HSG_E_INVALID;
  const uint64_t n = j->pending;
  if (n) {
    JTRY(hipSetDevice(j->device));
    const hipMemcpyKind k = o->mem == HSG_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
    if (o->this_handle) JTRY(hipMemcpyAsync(o->this_handle, j->out.this_h, n * 8, k, j->stream));
    if (o->other_handle) JTRY(hipMemcpyAsync(o->other_handle, j->out.other_h, n * 8, k, j->stream));
    if (o->join_key) JTRY(hipMemcpyAsync(o->join_key, j->out.jkey, n * 4, k, j->stream));
    if (o->ts) JTRY(hipMemcpyAsync(o->ts, j->out.ts, n * 8, k, j->stream));
    JTRY(hipStreamSynchronize(j->stream));
  }
  j->pending = 0;
  return HSG_OK;
}
