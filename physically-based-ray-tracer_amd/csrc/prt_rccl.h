// prt_rccl.h -- RCCL entry points for the sharded contexts (include/prt.h, prt_shard_*), resolved at run time.
//
// libprt.so does not link RCCL: a process that never shards a frame never loads it.  The first shard call
// looks for an already-loaded librccl.so.1 (the one torch ships, when the host process imported torch) and
// only otherwise loads /opt/rocm's, so one process never holds two RCCL copies.  Only the calls the
// framebuffer gather needs are bound.
#pragma once
#include <rccl/rccl.h>

namespace prt {

struct Rccl {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*);
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int);
  ncclResult_t (*CommDestroy)(ncclComm_t);
  ncclResult_t (*CommCount)(const ncclComm_t, int*);
  ncclResult_t (*CommUserRank)(const ncclComm_t, int*);
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*);
  ncclResult_t (*Gather)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t);
  const char* (*GetErrorString)(ncclResult_t);
  ncclResult_t (*CommAbort)(ncclComm_t);  // optional (nullptr when the library lacks it)
  // optional: a non-blocking communicator (config.blocking = 0), so a rank whose peers never arrive can give up
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*);
};

// nullptr when RCCL cannot be loaded (the message is in *why)
const Rccl* rccl(const char** why);

}  // namespace prt
