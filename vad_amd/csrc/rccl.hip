// RCCL entry points of the C ABI (include/vad_amd.h, vad_rccl_*): the one
// collective of the multi-GPU clip path -- a gather of per-window uint8
// decisions to the root rank (rccl.h ncclGather) -- for hosts
// that drive libvad_amd.so without torch.distributed.  RCCL is resolved at
// run time: the copy already loaded in the process (torch's) if there is one,
// else the system librccl.so.1, so the library itself links no RCCL and a
// process never holds two communicator implementations by accident.
#include <dlfcn.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>

#include "vad_common.h"

namespace {

typedef int nccl_result;  // ncclResult_t (0 = ncclSuccess)
typedef void* nccl_comm;  // ncclComm_t
struct nccl_uid {
  char internal[VAD_RCCL_ID_BYTES];
};
constexpr int kNcclUint8 = 1;  // ncclDataType_t ncclUint8

struct Rccl {
  void* handle = nullptr;
  nccl_result (*get_unique_id)(nccl_uid*) = nullptr;
  nccl_result (*comm_init_rank)(nccl_comm*, int, nccl_uid, int) = nullptr;
  nccl_result (*gather)(const void*, void*, size_t, int, int, nccl_comm, hipStream_t) = nullptr;
  nccl_result (*comm_destroy)(nccl_comm) = nullptr;
  const char* (*error_string)(nccl_result) = nullptr;
};

Rccl g_rccl;
std::once_flag g_once;
thread_local char g_err[256] = "";

void load_rccl() {
  void* h = nullptr;
  for (const char* name : {"librccl.so.1", "librccl.so"})
    if (!h) h = dlopen(name, RTLD_NOW | RTLD_LOCAL | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
  if (!h) return;
  Rccl r;
  r.handle = h;
  r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
  r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
  r.gather = reinterpret_cast<decltype(r.gather)>(dlsym(h, "ncclGather"));
  r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
  r.error_string = reinterpret_cast<decltype(r.error_string)>(dlsym(h, "ncclGetErrorString"));
  if (r.get_unique_id && r.comm_init_rank && r.gather && r.comm_destroy) g_rccl = r;
}

const Rccl* rccl() {
  std::call_once(g_once, load_rccl);
  return g_rccl.handle && g_rccl.gather ? &g_rccl : nullptr;
}

int fail(const Rccl* r, nccl_result e) {
  const char* msg = r && r->error_string ? r->error_string(e) : "RCCL error";
  strncpy(g_err, msg ? msg : "RCCL error", sizeof(g_err) - 1);
  return VAD_ERCCL;
}

}  // namespace

struct vad_rccl_comm {
  nccl_comm comm;
  int nranks;
  int rank;
};

extern "C" {

int vad_rccl_available(void) { return rccl() != nullptr; }

const char* vad_rccl_error_string(void) { return g_err; }

int vad_rccl_unique_id(void* id) {
  if (!id) return VAD_EINVAL;
  const Rccl* r = rccl();
  if (!r) return VAD_EUNSUPPORTED;
  nccl_uid u;
  const nccl_result e = r->get_unique_id(&u);
  if (e) return fail(r, e);
  memcpy(id, &u, sizeof(u));
  return VAD_OK;
}

int vad_rccl_init(vad_rccl_comm** out, int32_t nranks, const void* id, int32_t rank) {
  if (!out || !id || nranks <= 0 || rank < 0 || rank >= nranks) return VAD_EINVAL;
  const Rccl* r = rccl();
  if (!r) return VAD_EUNSUPPORTED;
  nccl_uid u;
  memcpy(&u, id, sizeof(u));
  nccl_comm c = nullptr;
  const nccl_result e = r->comm_init_rank(&c, nranks, u, rank);  // on the current HIP device
  if (e) return fail(r, e);
  vad_rccl_comm* p = (vad_rccl_comm*)calloc(1, sizeof(vad_rccl_comm));
  if (!p) {
    r->comm_destroy(c);
    return VAD_ENOMEM;
  }
  p->comm = c;
  p->nranks = nranks;
  p->rank = rank;
  *out = p;
  return VAD_OK;
}

int vad_rccl_gather_u8(vad_rccl_comm* comm, const uint8_t* send, uint8_t* recv, size_t count, int32_t root,
                       void* stream) {
  if (!comm || root < 0 || root >= comm->nranks) return VAD_EINVAL;
  if (count == 0) return VAD_OK;
  if (!send || (comm->rank == root && !recv)) return VAD_EINVAL;
  const Rccl* r = rccl();
  if (!r) return VAD_EUNSUPPORTED;
  const nccl_result e = r->gather(send, recv, count, kNcclUint8, root, comm->comm, (hipStream_t)stream);
  return e ? fail(r, e) : VAD_OK;
}

int vad_rccl_destroy(vad_rccl_comm* comm) {
  if (!comm) return VAD_OK;
  const Rccl* r = rccl();
  int rc = VAD_OK;
  if (r) {
    const nccl_result e = r->comm_destroy(comm->comm);
    if (e) rc = fail(r, e);
  }
  free(comm);
  return rc;
}

}  // extern "C"
