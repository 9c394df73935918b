// RCCL loaded at run time (rccl_dyn.h) and the communicator helpers of the C ABI
// (acme_nccl_*), for callers of the data-parallel learner that bring no communicator.
#include "rccl_dyn.h"

#include <dlfcn.h>

#include <cstring>
#include <mutex>

#include "common.h"

namespace acme {
namespace rccl {

const Api* api() {
  static std::once_flag once;
  static Api a;
  static bool ok = false;
  std::call_once(once, [] {
    // A copy already in the process first (torch's), then the system one.
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so"}) {
      h = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
      if (h) break;
    }
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      if (h) break;
      h = dlopen(name, RTLD_NOW | RTLD_GLOBAL);
    }
    if (!h) return;
    a.GetUniqueId = reinterpret_cast<decltype(a.GetUniqueId)>(dlsym(h, "ncclGetUniqueId"));
    a.CommInitRank = reinterpret_cast<decltype(a.CommInitRank)>(dlsym(h, "ncclCommInitRank"));
    a.CommDestroy = reinterpret_cast<decltype(a.CommDestroy)>(dlsym(h, "ncclCommDestroy"));
    a.AllReduce = reinterpret_cast<decltype(a.AllReduce)>(dlsym(h, "ncclAllReduce"));
    a.GetErrorString =
        reinterpret_cast<decltype(a.GetErrorString)>(dlsym(h, "ncclGetErrorString"));
    ok = a.GetUniqueId && a.CommInitRank && a.CommDestroy && a.AllReduce && a.GetErrorString;
  });
  if (!ok) {
    set_error("RCCL (librccl.so.1) could not be loaded");
    return nullptr;
  }
  return &a;
}

}  // namespace rccl
}  // namespace acme

using acme::set_error;

extern "C" {

int acme_nccl_get_unique_id(uint8_t* out) {
  ACME_CHECK_ARG(out, "null argument");
  const acme::rccl::Api* r = acme::rccl::api();
  if (!r) return ACME_ERR_HIP;
  ncclUniqueId id;
  const ncclResult_t e = r->GetUniqueId(&id);
  if (e != ncclSuccess) {
    set_error("ncclGetUniqueId: %s", r->GetErrorString(e));
    return ACME_ERR_HIP;
  }
  std::memcpy(out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return ACME_OK;
}

int acme_nccl_comm_init(const uint8_t* id, int32_t world_size, int32_t rank, void** comm) {
  ACME_CHECK_ARG(id && comm && world_size >= 1 && rank >= 0 && rank < world_size,
                 "bad communicator arguments");
  const acme::rccl::Api* r = acme::rccl::api();
  if (!r) return ACME_ERR_HIP;
  ncclUniqueId uid;
  std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t c = nullptr;
  const ncclResult_t e = r->CommInitRank(&c, world_size, uid, rank);
  if (e != ncclSuccess) {
    set_error("ncclCommInitRank: %s", r->GetErrorString(e));
    return ACME_ERR_HIP;
  }
  *comm = c;
  return ACME_OK;
}

int acme_nccl_comm_destroy(void* comm) {
  if (!comm) return ACME_OK;
  const acme::rccl::Api* r = acme::rccl::api();
  if (!r) return ACME_ERR_HIP;
  const ncclResult_t e = r->CommDestroy(static_cast<ncclComm_t>(comm));
  if (e != ncclSuccess) {
    set_error("ncclCommDestroy: %s", r->GetErrorString(e));
    return ACME_ERR_HIP;
  }
  return ACME_OK;
}

}  // extern "C"
