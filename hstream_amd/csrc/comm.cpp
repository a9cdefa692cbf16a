// RCCL communicator owned by the engine (one per process and GPU).
#include <cstring>
#include <string>

#include "hsg_exchange.h"
#include "hsg_kernels.h"

namespace hsg {

static_assert(sizeof(ncclUniqueId) <= HSG_COMM_ID_BYTES, "ncclUniqueId larger than HSG_COMM_ID_BYTES");

int comm_unique_id(uint8_t *out) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return HSG_E_COMM;
  memset(out, 0, HSG_COMM_ID_BYTES);
  memcpy(out, &id, sizeof(id));
  return HSG_OK;
}

int comm_create(const uint8_t *id_bytes, int rank, int nranks, int device, Comm **out, std::string &err) {
  if (nranks > kMaxRanks) {
    err = "too many ranks";
    return HSG_E_INVALID;
  }
  ncclUniqueId id;
  memcpy(&id, id_bytes, sizeof(id));
  Comm *c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    err = std::string("ncclCommInitRank: ") + ncclGetErrorString(r);
    delete c;
    return HSG_E_COMM;
  }
  *out = c;
  return HSG_OK;
}

// A communicator of the same ranks for one operator (collective over the
// parent's ranks, so every rank calls it in the same op-creation order).
int comm_split(const Comm *parent, Comm **out, std::string &err) {
  Comm *c = new Comm();
  c->rank = parent->rank;
  c->nranks = parent->nranks;
  ncclResult_t r = ncclCommSplit(parent->comm, 0, parent->rank, &c->comm, nullptr);
  if (r != ncclSuccess) {
    err = std::string("ncclCommSplit: ") + ncclGetErrorString(r);
    delete c;
    return HSG_E_COMM;
  }
  *out = c;
  return HSG_OK;
}

void comm_destroy(Comm *c) {
  if (!c) return;
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
}

}  // namespace hsg
