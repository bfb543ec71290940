// RCCL (over xGMI): the one real exchange step of data-parallel log_prob —
// the all-reduce of the fp64 NLL partial sums (train.py:75-78 defines the NLL;
// SURVEY.md §8e) — and the all-gather behind data-parallel training
// (zf_trainer_set_comm).  librccl is dlopen'ed lazily so loading libzenflow_amd.so
// never pulls RCCL into processes that do not need it.
#include <dlfcn.h>

#include <cstring>

#include <rccl/rccl.h>

#include "zf_internal.h"

namespace zf {
namespace {

struct Rccl {
  void* lib = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool tried = false;
};

Rccl& rccl() {
  static Rccl r;
  if (!r.tried) {
    r.tried = true;
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names) {
      r.lib = dlopen(n, RTLD_NOW | RTLD_LOCAL);
      if (r.lib) break;
    }
    if (r.lib) {
      r.get_unique_id = (decltype(r.get_unique_id))dlsym(r.lib, "ncclGetUniqueId");
      r.comm_init_rank = (decltype(r.comm_init_rank))dlsym(r.lib, "ncclCommInitRank");
      r.all_reduce = (decltype(r.all_reduce))dlsym(r.lib, "ncclAllReduce");
      r.all_gather = (decltype(r.all_gather))dlsym(r.lib, "ncclAllGather");
      r.comm_destroy = (decltype(r.comm_destroy))dlsym(r.lib, "ncclCommDestroy");
      r.error_string = (decltype(r.error_string))dlsym(r.lib, "ncclGetErrorString");
    }
  }
  return r;
}

int nccl_status(ncclResult_t e, const char* what) {
  if (e == ncclSuccess) return ZF_OK;
  const char* msg = rccl().error_string ? rccl().error_string(e) : "?";
  set_error("%s: %s (%d)", what, msg, (int)e);
  return 1000 + (int)e;
}

bool loaded() {
  Rccl& r = rccl();
  return r.get_unique_id && r.comm_init_rank && r.all_reduce && r.all_gather && r.comm_destroy;
}

}  // namespace
}  // namespace zf

extern "C" {

int zf_rccl_available(void) { return zf::loaded() ? 1 : 0; }

int zf_rccl_get_unique_id(char* id128) {
  if (!zf::loaded()) { zf::set_error("librccl not available"); return ZF_ENOTSUP; }
  if (!id128) return zf::einval("id is NULL");
  ncclUniqueId id;
  int rc = zf::nccl_status(zf::rccl().get_unique_id(&id), "ncclGetUniqueId");
  if (rc) return rc;
  std::memcpy(id128, id.internal, NCCL_UNIQUE_ID_BYTES);
  return ZF_OK;
}

int zf_rccl_comm_init(void** comm, int nranks, const char* id128, int rank) {
  if (!zf::loaded()) { zf::set_error("librccl not available"); return ZF_ENOTSUP; }
  if (!comm || !id128) return zf::einval("NULL argument");
  ncclUniqueId id;
  std::memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c;
  int rc = zf::nccl_status(zf::rccl().comm_init_rank(&c, nranks, id, rank), "ncclCommInitRank");
  if (rc) return rc;
  *comm = (void*)c;
  return ZF_OK;
}

int zf_rccl_allreduce_sum_f64(void* comm, const double* send, double* recv, size_t count,
                              void* stream) {
  if (!zf::loaded()) { zf::set_error("librccl not available"); return ZF_ENOTSUP; }
  return zf::nccl_status(zf::rccl().all_reduce(send, recv, count, ncclFloat64, ncclSum,
                                                (ncclComm_t)comm, (hipStream_t)stream),
                         "ncclAllReduce");
}

int zf_rccl_allgather(void* comm, const void* send, void* recv, size_t bytes, void* stream) {
  if (!zf::loaded()) { zf::set_error("librccl not available"); return ZF_ENOTSUP; }
  return zf::nccl_status(zf::rccl().all_gather(send, recv, bytes, ncclInt8, (ncclComm_t)comm, (hipStream_t)stream),
                         "ncclAllGather");
}

int zf_rccl_comm_destroy(void* comm) {
  if (!comm) return ZF_OK;
  if (!zf::loaded()) return ZF_OK;
  return zf::nccl_status(zf::rccl().comm_destroy((ncclComm_t)comm), "ncclCommDestroy");
}

}  // extern "C"
