// RCCL entry points resolved at run time (dlopen), so libacme_hip.so loads without RCCL and
// shares the process's copy when one is already loaded (torch's ProcessGroupNCCL).  Only
// the data-parallel entry points (acme_dqn_dp_*, acme_nccl_*) need it.
#pragma once

#include <rccl/rccl.h>

namespace acme {
namespace rccl {

struct Api {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                            hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

// The loaded API, or nullptr (with acme_last_error set) if RCCL cannot be found.
const Api* api();

}  // namespace rccl
}  // namespace acme
