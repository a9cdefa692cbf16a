// Communicators of the key exchange (exchange.cpp): RCCL (one process per
// GPU, xGMI on an MI355X node) or, for tests of several ranks on one host and
// GPU, a shared-memory transport with the same collectives.
#include <fcntl.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "hsg_exchange.h"
#include "hsg_kernels.h"

namespace hsg {

static_assert(sizeof(ncclUniqueId) <= HSG_COMM_ID_BYTES, "ncclUniqueId larger than HSG_COMM_ID_BYTES");

// ---------------------------------------------------------------------------
// shared-memory transport (HSG_TRANSPORT_HOST)
// ---------------------------------------------------------------------------
// One POSIX shared-memory segment per communicator, named by the caller's id
// (split communicators append their split number: every rank splits in the
// same order). Layout: a control line (barrier counter, generation), then one
// slot per rank: [scount[kMaxRanks]][sdispl[kMaxRanks]][data]. A collective
// copies the rank's device data into its slot, meets the others at a barrier,
// copies what it receives out of their slots, and meets them again before the
// slots are reused. Device data produced on the op's stream is synchronised
// first; the copies back are synchronous, so later work on the stream sees them.
struct HostComm {
  std::string name;
  int rank = 0, nranks = 1;
  size_t slot_data = 0;   // data bytes per rank slot
  size_t bytes = 0;
  char *base = nullptr;
  int splits = 0;
};

constexpr size_t kCtrl = 256;
constexpr size_t kSlotHdr = 2 * kMaxRanks * sizeof(uint64_t);

static uint32_t *ctl_count(HostComm *h) { return (uint32_t *)h->base; }
static uint32_t *ctl_gen(HostComm *h) { return (uint32_t *)(h->base + 64); }
// set once a barrier timed out or a collective's ranks disagreed: the
// communicator is dead, every later barrier on it fails at once on every rank
// (a timed-out rank's arrival stays in the counter, so the generations no
// longer line up)
static uint32_t *ctl_failed(HostComm *h) { return (uint32_t *)(h->base + 128); }
static int host_fail(HostComm *h, std::string &err, const std::string &why) {
  __atomic_store_n(ctl_failed(h), 1u, __ATOMIC_RELEASE);
  err = why;
  return HSG_E_COMM;
}
static char *slot(HostComm *h, int r) { return h->base + kCtrl + (size_t)r * (kSlotHdr + h->slot_data); }

// centralised barrier over the segment's counter; a peer that never arrives
// (crashed) ends it with an error after a minute instead of hanging
static int host_barrier(HostComm *h, std::string &err) {
  if (__atomic_load_n(ctl_failed(h), __ATOMIC_ACQUIRE)) {
    err = "host transport: the communicator failed earlier (a rank timed out or disagreed)";
    return HSG_E_COMM;
  }
  const uint32_t gen = __atomic_load_n(ctl_gen(h), __ATOMIC_ACQUIRE);
  const uint32_t arrived = __atomic_add_fetch(ctl_count(h), 1u, __ATOMIC_ACQ_REL);
  if (arrived == (uint32_t)h->nranks) {
    __atomic_store_n(ctl_count(h), 0u, __ATOMIC_RELAXED);
    __atomic_store_n(ctl_gen(h), gen + 1, __ATOMIC_RELEASE);
    return HSG_OK;
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 0; __atomic_load_n(ctl_gen(h), __ATOMIC_ACQUIRE) == gen; ++spin) {
    if ((spin & 1023) == 0) {
      sched_yield();
      if (__atomic_load_n(ctl_failed(h), __ATOMIC_ACQUIRE))
        return host_fail(h, err, "host transport: a peer rank failed the collective");
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60))
        return host_fail(h, err, "host transport: a peer rank did not reach the barrier within 60 s");
    }
  }
  return HSG_OK;
}

static int host_open(const std::string &name, int rank, int nranks, size_t slot_data, HostComm **out,
                     std::string &err) {
  HostComm *h = new HostComm();
  h->name = name;
  h->rank = rank;
  h->nranks = nranks;
  h->slot_data = (slot_data + 255) & ~(size_t)255;
  h->bytes = kCtrl + (size_t)nranks * (kSlotHdr + h->slot_data);
  const std::string path = "/" + name;
  const int fd = shm_open(path.c_str(), O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, (off_t)h->bytes) != 0) {
    if (fd >= 0) close(fd);
    err = "host transport: shm_open / ftruncate " + path + " failed";
    delete h;
    return HSG_E_COMM;
  }
  void *p = mmap(nullptr, h->bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    err = "host transport: mmap failed";
    delete h;
    return HSG_E_COMM;
  }
  h->base = (char *)p;
  // every rank has mapped the segment: its name can go (no file outlives a crash)
  int rc = host_barrier(h, err);
  if (rc == HSG_OK && rank == 0) shm_unlink(path.c_str());
  if (rc != HSG_OK) {
    munmap(h->base, h->bytes);
    delete h;
    return rc;
  }
  *out = h;
  return HSG_OK;
}

static void host_close(HostComm *h) {
  if (!h) return;
  if (h->base) munmap(h->base, h->bytes);
  delete h;
}

// ---------------------------------------------------------------------------
// communicators
// ---------------------------------------------------------------------------
int comm_unique_id(uint8_t *out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return HSG_E_COMM;
  memset(out, 0, HSG_COMM_ID_BYTES);
  memcpy(out, &id, sizeof(id));
  return HSG_OK;
}

// comm_agree's stream and buffer, made with the communicator so that a rank
// whose op creation fails later still reaches the agreement without
// allocating anything
static int agree_alloc(Comm *c, std::string &err) {
  if (hipStreamCreateWithFlags(&c->agree_s, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void **)&c->agree_buf, ((size_t)c->nranks + 1) * sizeof(int64_t)) != hipSuccess) {
    err = "communicator: agreement stream / buffer";
    return HSG_E_DEVICE;
  }
  return HSG_OK;
}

int comm_create(const uint8_t *id_bytes, int rank, int nranks, int device, int transport, uint64_t batch_cap,
                Comm **out, std::string &err) {
  if (nranks > kMaxRanks) {
    err = "too many ranks";
    return HSG_E_INVALID;
  }
  Comm *c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  if (transport == HSG_TRANSPORT_HOST) {
    char name[HSG_COMM_ID_BYTES + 1];
    memcpy(name, id_bytes, HSG_COMM_ID_BYTES);
    name[HSG_COMM_ID_BYTES] = 0;
    if (!name[0] || strchr(name, '/')) {
      err = "host transport: comm_id must be a NUL-terminated name without '/'";
      delete c;
      return HSG_E_INVALID;
    }
    // the largest collective: the classic exchange's packed records (<= 12 words each)
    c->slot_bytes = batch_cap * 12 * 8 + 4096;
    // the rendezvous first, whatever the allocation below does: no rank
    // skips a collective its peers have entered
    int rc = host_open(name, rank, nranks, c->slot_bytes, &c->host, err);
    std::string aerr;
    const int arc = agree_alloc(c, aerr);
    if (rc == HSG_OK && arc != HSG_OK) {
      rc = arc;
      err = aerr;
    }
    if (rc != HSG_OK) {
      comm_destroy(c);
      return rc;
    }
    *out = c;
    return HSG_OK;
  }
  // the communicator init first, whatever the allocation of the agreement
  // buffer does: every rank joins the collective init (a rank that returned
  // before it would leave its peers waiting there). A rank whose 16-byte
  // agreement buffer then fails to allocate returns the error; its peers see
  // it at their first agreement (op creation), which that rank never joins --
  // the caller must not go on with the engine on any rank then.
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  const ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  std::string aerr;
  const int arc = agree_alloc(c, aerr);
  if (r != ncclSuccess) {
    err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    comm_destroy(c);
    return HSG_E_COMM;
  }
  if (arc != HSG_OK) {
    err = aerr;
    comm_destroy(c);
    return arc;
  }
  *out = c;
  return HSG_OK;
}

// A communicator of the same ranks for one operator (collective over the
// parent's ranks, so every rank calls it in the same op-creation order).
// The split is collective over the parent's ranks, and so is its outcome:
// every rank allocates the child's agreement buffer first (nothing collective
// yet), takes part in the split whatever that allocation did, and then the
// ranks agree on the parent -- whose agreement buffer exists since the engine
// was created -- so that a failure on one rank (its allocation or its split)
// fails the split on every rank, and no rank goes on to a collective of the
// child that a peer never reaches. Callers serialize splits of one parent
// (hsg_op_create holds the engine's lock), which the parent's one agreement
// buffer needs.
int comm_split(Comm *parent, Comm **out, std::string &err) {
  *out = nullptr;
  Comm *c = new Comm();
  c->rank = parent->rank;
  c->nranks = parent->nranks;
  std::string lerr;
  int rc = agree_alloc(c, lerr);
  if (parent->host) {
    c->slot_bytes = parent->slot_bytes;
    const std::string name = parent->host->name + "." + std::to_string(++parent->host->splits);
    const int src = host_open(name, c->rank, c->nranks, c->slot_bytes, &c->host, lerr);
    if (rc == HSG_OK) rc = src;
  } else {
    const ncclResult_t r = ncclCommSplit(parent->comm, 0, parent->rank, &c->comm, nullptr);
    if (r != ncclSuccess && rc == HSG_OK) {
      lerr = std::string("ncclCommSplit: ") + ncclGetErrorString(r);
      rc = HSG_E_COMM;
    }
  }
  std::string aerr;
  const int arc = comm_agree(parent, rc, aerr);
  if (rc != HSG_OK || arc != HSG_OK) {
    err = rc != HSG_OK ? lerr : aerr;
    comm_destroy(c);
    return rc != HSG_OK ? rc : arc;
  }
  *out = c;
  return HSG_OK;
}

void comm_destroy(Comm *c) {
  if (!c) return;
  if (c->agree_buf) hipFree(c->agree_buf);
  if (c->agree_s) hipStreamDestroy(c->agree_s);
  if (c->comm) ncclCommDestroy(c->comm);
  host_close(c->host);
  delete c;
}

#define CNTRY(expr)                                                         \
  do {                                                                      \
    ncclResult_t _r = (expr);                                               \
    if (_r != ncclSuccess) {                                                \
      err = std::string(#expr) + ": " + ncclGetErrorString(_r);             \
      return HSG_E_COMM;                                                    \
    }                                                                       \
  } while (0)
#define CHTRY(expr)                                                         \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) {                                                 \
      err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return HSG_E_DEVICE;                                                  \
    }                                                                       \
  } while (0)

int comm_group_start(Comm *c, std::string &err) {
  if (!c->host) CNTRY(ncclGroupStart());
  return HSG_OK;
}

int comm_group_end(Comm *c, std::string &err) {
  if (!c->host) CNTRY(ncclGroupEnd());
  return HSG_OK;
}

int comm_allgather(Comm *c, const void *send, void *recv, size_t count, ncclDataType_t dt, size_t elem,
                   hipStream_t s, std::string &err) {
  if (!c->host) {
    CNTRY(ncclAllGather(send, recv, count, dt, c->comm, s));
    return HSG_OK;
  }
  HostComm *h = c->host;
  const size_t bytes = count * elem;
  if (bytes > h->slot_data) {
    err = "host transport: all-gather larger than a slot";
    return HSG_E_COMM;
  }
  CHTRY(hipStreamSynchronize(s));
  CHTRY(hipMemcpy(slot(h, h->rank) + kSlotHdr, send, bytes, hipMemcpyDeviceToHost));
  int rc = host_barrier(h, err);
  if (rc != HSG_OK) return rc;
  for (int q = 0; q < h->nranks; ++q)
    CHTRY(hipMemcpy((char *)recv + (size_t)q * bytes, slot(h, q) + kSlotHdr, bytes, hipMemcpyHostToDevice));
  return host_barrier(h, err);
}

// Every rank's status of a collective step (op creation): one all-gather of
// an int64 per rank. Returns the first failing rank's code (HSG_OK when all
// succeeded), or the transport's own error.
int comm_agree(Comm *c, int rc_local, std::string &err) {
  hipStream_t s = c->agree_s;
  int64_t *buf = c->agree_buf;
  std::vector<int64_t> h((size_t)c->nranks + 1, 0);
  h[0] = rc_local;
  int rc = HSG_OK;
  if (!s || !buf) {
    err = "comm_agree: no agreement buffer (communicator setup failed)";
    return HSG_E_DEVICE;
  }
  // every step below runs even after a local failure: a rank that skipped
  // the all-gather would leave its peers waiting in it
  hipError_t e = hipMemcpyAsync(buf, h.data(), sizeof(int64_t), hipMemcpyHostToDevice, s);
  if (e != hipSuccess) {
    err = std::string("comm_agree: ") + hipGetErrorString(e);
    rc = HSG_E_DEVICE;
  }
  const int grc = comm_allgather(c, buf, buf + 1, 1, ncclInt64, sizeof(int64_t), s, err);
  if (rc == HSG_OK) rc = grc;
  if (rc == HSG_OK) {
    e = hipMemcpyAsync(h.data() + 1, buf + 1, (size_t)c->nranks * sizeof(int64_t), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
      err = std::string("comm_agree: ") + hipGetErrorString(e);
      rc = HSG_E_DEVICE;
    }
  }
  if (rc == HSG_OK)
    for (int q = 0; q < c->nranks; ++q)
      if (h[1 + q] != HSG_OK) {
        if (rc_local == HSG_OK) err = "rank " + std::to_string(q) + " failed to create its shard of the operator";
        rc = (int)h[1 + q];
        break;
      }
  return rc;
}

int comm_alltoallv(Comm *c, const void *send, const size_t *scount, const size_t *sdispl, void *recv,
                   const size_t *rcount, const size_t *rdispl, ncclDataType_t dt, size_t elem, hipStream_t s,
                   std::string &err) {
  if (!c->host) {
    CNTRY(ncclAllToAllv(send, scount, sdispl, recv, rcount, rdispl, dt, c->comm, s));
    return HSG_OK;
  }
  HostComm *h = c->host;
  const int G = h->nranks, me = h->rank;
  size_t total = 0;
  for (int q = 0; q < G; ++q) total = sdispl[q] + scount[q] > total ? sdispl[q] + scount[q] : total;
  if (total * elem > h->slot_data) {
    err = "host transport: all-to-all larger than a slot";
    return HSG_E_COMM;
  }
  CHTRY(hipStreamSynchronize(s));
  uint64_t *hdr = (uint64_t *)slot(h, me);
  for (int q = 0; q < G; ++q) {
    hdr[q] = scount[q];
    hdr[kMaxRanks + q] = sdispl[q];
  }
  if (total) CHTRY(hipMemcpy(slot(h, me) + kSlotHdr, send, total * elem, hipMemcpyDeviceToHost));
  int rc = host_barrier(h, err);
  if (rc != HSG_OK) return rc;
  for (int q = 0; q < G; ++q) {
    const uint64_t *ph = (const uint64_t *)slot(h, q);
    if (ph[me] != rcount[q])  // every waiter sees the flag: no rank is left in a barrier
      return host_fail(h, err, "host transport: all-to-all counts disagree");
    if (rcount[q])
      CHTRY(hipMemcpy((char *)recv + rdispl[q] * elem, slot(h, q) + kSlotHdr + ph[kMaxRanks + me] * elem,
                      rcount[q] * elem, hipMemcpyHostToDevice));
  }
  return host_barrier(h, err);
}

}  // namespace hsg
