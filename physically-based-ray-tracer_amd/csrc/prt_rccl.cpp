// prt_rccl.cpp -- run-time binding of the RCCL calls the sharded frame gather uses (prt_rccl.h).
#include "prt_rccl.h"

#include <dlfcn.h>

#include <mutex>

namespace prt {

namespace {

Rccl g_rccl;
const Rccl* g_ok = nullptr;
const char* g_why = "RCCL not loaded";
std::once_flag g_once;

template <class F>
bool bind(void* h, F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(h, name));
  return f != nullptr;
}

void load() {
  // the copy the process already holds (torch's), else the ROCm install's
  void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
  if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
  if (!h) {
    g_why = "librccl.so.1 could not be loaded";
    return;
  }
  Rccl& r = g_rccl;
  if (!bind(h, r.GetUniqueId, "ncclGetUniqueId") || !bind(h, r.CommInitRank, "ncclCommInitRank") ||
      !bind(h, r.CommDestroy, "ncclCommDestroy") || !bind(h, r.CommCount, "ncclCommCount") ||
      !bind(h, r.CommUserRank, "ncclCommUserRank") || !bind(h, r.CommGetAsyncError, "ncclCommGetAsyncError") ||
      !bind(h, r.Gather, "ncclGather") || !bind(h, r.GetErrorString, "ncclGetErrorString")) {
    g_why = "librccl.so.1 lacks a required entry point (ncclGather needs RCCL >= 2.18)";
    return;
  }
  r.CommAbort = reinterpret_cast<ncclResult_t (*)(ncclComm_t)>(dlsym(h, "ncclCommAbort"));
  r.CommInitRankConfig = reinterpret_cast<ncclResult_t (*)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*)>(
      dlsym(h, "ncclCommInitRankConfig"));
  g_ok = &g_rccl;
}

}  // namespace

const Rccl* rccl(const char** why) {
  std::call_once(g_once, load);
  if (!g_ok && why) *why = g_why;
  return g_ok;
}

}  // namespace prt
