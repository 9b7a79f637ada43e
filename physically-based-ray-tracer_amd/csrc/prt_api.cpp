// prt_api.cpp -- C-ABI implementation (include/prt.h): device residency of the scene, BLAS build,
// kernel orchestration.  One host thread per context; all device work on one HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/prt.h"
#include "bvh_build.h"
#include "bvh_gpu.h"
#include "prt_launch.h"
#include "prt_rccl.h"
#include "prt_refit.h"

using namespace prt;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) return fail(PRT_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

// device allocation owned by its holder (move-only; freed on destruction)
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), bytes(o.bytes) { o.p = nullptr; o.bytes = 0; }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) { release(); p = o.p; bytes = o.bytes; o.p = nullptr; o.bytes = 0; }
    return *this;
  }
  ~DevBuf() { release(); }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  // (re)allocate to at least n bytes; contents are not preserved
  hipError_t ensure(size_t n) {
    if (n <= bytes && p) return hipSuccess;
    release();
    hipError_t e = hipMalloc(&p, n ? n : 16);
    if (e == hipSuccess) bytes = n ? n : 16;
    return e;
  }
  template <class T>
  T* as() const { return reinterpret_cast<T*>(p); }
};

// blocking host -> device copy into a resident buffer.  Callers that may overwrite (or reallocate) a buffer
// that queued frames still read first drain the context stream (drain()).
hipError_t upload(DevBuf& b, const void* src, size_t n) {
  hipError_t e = b.ensure(n);
  if (e != hipSuccess) return e;
  if (n) return hipMemcpy(b.p, src, n, hipMemcpyHostToDevice);
  return hipSuccess;
}


// wavefront state of one item group: the context's own (prt_ctx::ws), or of a concurrent group (prt_ctx::grp)
struct WaveState {
  DevBuf wave;
  WaveBufs wb = {};
  uint32_t n = 0, levels = 0;
  bool ext = false, merge = false;
};
// a frame in flight (prt_set_frames_in_flight): the wavefront chain of one call on its own stream.  Slot 0 uses the
// context's own wavefront state and frame buffer, the others their own; done = the call's last work (the
// accumulation, and for a sharded frame its gather and untile), which the next call's accumulation waits for
constexpr int kMaxFlights = 8;
struct Flight {
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  WaveState ws;
  DevBuf frames;
  bool pending = false;  // done is not yet in the context stream's order
};

// one pinned staging buffer of ensure_instances' uploads (prt_ctx::stage): reused once its copies have run.  The
// kStageSlots buffers are allocated when an instance set is first built (pinned allocation in the update path cost
// 20-190 ms per buffer on the GPU box, profiles/r06_tlas_drift.txt); an update that finds all of them in use waits
// for the oldest one's copies (the host at most kStageSlots updates ahead of the GPU)
constexpr size_t kStageSlots = 8;
// the stream's wait for a worker build: a build takes ~6 ms at 10,000 instances and the jobs of up to kStageSlots
// queued updates run one after another, so the limit only catches a producer that never comes
constexpr double kHostWaitLimitS = 120.0;
struct StageSlot {
  void* p = nullptr;
  size_t bytes = 0;
  hipEvent_t ev = nullptr;
  bool used = false;
  bool lost = false;  // an update failed while enqueuing from it: never handed out again (its copies may be pending)
  uint64_t seq = 0;   // when it was last acquired
};
// One copy of the instance state the frames read (prt_ctx::isets): instance records, their refit input, the instance
// BVH.  An update writes the next copy in the ring while the frames in flight still read theirs; a copy is
// rewritten only after the context stream has waited for the frames that read it (one event per stream they ran on)
struct InstSet {
  DevBuf inst, inst_src, tlas8, tlas_slot;
  std::vector<std::pair<hipStream_t, hipEvent_t>> uses;  // the last frame that read this copy, per stream
  size_t nuse = 0;
};
// The instance BVH's per-update build (ensure_instances) on the context's worker thread: each update's job builds
// the tree over that update's instance boxes into the update's pinned staging buffer, then sets the update's flag
// word; the render stream waits for the flag in a one-lane kernel (launch_wait_host) placed before the tree's
// upload, so the calling thread never builds nor waits, and the frames already queued run while the worker builds.
// (A host function, hipLaunchHostFunc, made the next enqueue on the stream block the calling thread until it had
// run: 5-11 ms per update with frames queued, scripts/inst_update_probe.py.)  Jobs run in submission order and every
// job sets its flag, also when its build fails; the worker never calls HIP.
struct TlasJob {
  const InstSrc* src = nullptr;  // the update's instances (in its pinned staging buffer, uploaded before the tree)
  int32_t n = 0;
  char* dst = nullptr;           // pinned: cap Node8 records, then 8 * cap slot words
  size_t cap = 0;                // nodes the upload moves (a tree over n instances has at most max(n, 1) nodes)
  int max_depth = 0;             // levels the traversal stacks were sized for (build_tlas8's cap)
  uint32_t* flag = nullptr;      // coherent pinned word: set to 1 once dst holds the tree
};
class TlasWorker {
 public:
  TlasWorker() : th_([this] { run(); }) {}
  ~TlasWorker() {  // after the streams are synchronised: the queue is empty (every job's stream wait has ended)
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    th_.join();
  }
  void seed(const BuiltTlas8& t) {  // the tree a failed build falls back to (its instance set's first tree)
    std::lock_guard<std::mutex> g(m_);
    good_nodes_ = t.nodes;
    good_slot_ = t.slot;
  }
  void submit(const std::shared_ptr<TlasJob>& j) {
    {
      std::lock_guard<std::mutex> g(m_);
      q_.push_back(j);
    }
    cv_.notify_all();
  }
  // diagnostics of the finished jobs
  struct Stats { double ms = 0, cpu_ms = 0; int32_t median = 0, failed = 0; std::string err; };
  Stats stats() {
    std::lock_guard<std::mutex> g(m_);
    return st_;
  }

 private:
  void run() {
    for (;;) {
      std::shared_ptr<TlasJob> j;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;  // stop_ with nothing queued
        j = q_.front();
        q_.pop_front();
      }
      const auto t0 = std::chrono::steady_clock::now();
      timespec c0{}, c1{};
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
      bool median = false, ok = false;
      std::string err;
      BuiltTlas8 t;
      try {  // the instances' world boxes (the same refit_instance as k_refit), the SAH build over them
        const int32_t m = j->n;
        std::vector<float> boxes(6 * (size_t)m);
        for (int32_t i = 0; i < m; i++) {
          InstDev I;
          refit_instance(j->src[i], I);
          std::memcpy(&boxes[6 * (size_t)i], I.bmin, 12);
          std::memcpy(&boxes[6 * (size_t)i + 3], I.bmax, 12);
        }
        t = build_tlas8(boxes.data(), m, j->max_depth);
        median = t.median;
        ok = t.nodes.size() <= j->cap && t.depth <= j->max_depth;
        if (!ok) err = "instance BVH larger than planned";
      } catch (const std::exception& e) {
        err = e.what();
      }
      std::lock_guard<std::mutex> g(m_);
      const std::vector<Node8>& nodes = ok ? t.nodes : good_nodes_;  // failed: the last good tree (valid links)
      const std::vector<uint32_t>& slot = ok ? t.slot : good_slot_;
      std::memcpy(j->dst, nodes.data(), std::min(nodes.size(), j->cap) * sizeof(Node8));
      std::memcpy(j->dst + j->cap * sizeof(Node8), slot.data(), std::min(slot.size(), 8 * j->cap) * 4);
      if (ok) {
        good_nodes_ = std::move(t.nodes);
        good_slot_ = std::move(t.slot);
      } else {
        st_.failed++;
        st_.err = err;
      }
      clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
      st_.ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      st_.cpu_ms = (c1.tv_sec - c0.tv_sec) * 1e3 + (c1.tv_nsec - c0.tv_nsec) * 1e-6;
      st_.median += median ? 1 : 0;
      __atomic_store_n(j->flag, 1u, __ATOMIC_RELEASE);  // the tree is in dst: the stream's wait ends
    }
  }
  std::mutex m_;
  std::condition_variable cv_;
  std::deque<std::shared_ptr<TlasJob>> q_;
  bool stop_ = false;
  std::vector<Node8> good_nodes_;
  std::vector<uint32_t> good_slot_;
  Stats st_;
  std::thread th_;  // last: started once the members above exist
};

struct MeshHost {
  float bmin[3], bmax[3];
  int depth;
  int64_t nodes, leaves;
  int32_t tris;
};

}  // namespace

struct prt_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  // textures
  std::vector<TexDev> tex_host;
  DevBuf texels, tex;
  // meshes
  std::vector<MeshDev> mesh_host;
  std::vector<MeshHost> mesh_info;
  DevBuf nodes8, tris, stri, mesh;
  int max_depth = 0;
  int builder = -1;  // BLAS builder (prt_set_bvh_builder): PRT_BUILDER_* (-1: PRT_BUILDER_HOST_SAH)
  double build_ms = 0;  // wall time of the last prt_set_meshes BLAS builds
  int built_with = PRT_BUILDER_HOST_SAH;
  // instances
  std::vector<float> inst_xf;
  std::vector<uint32_t> inst_mesh;
  std::vector<uint32_t> inst_kind;  // prt_set_instance_materials (PRT_MAT_*), textured by default
  std::vector<InstSrc> inst_stage;  // host side of the refit input (prt_refit.h)
  // the device instance state, one copy per frame in flight + 1 (InstSet); isets[icur] is what the next frame reads
  std::vector<InstSet> isets = std::vector<InstSet>(1);
  size_t icur = 0;
  // instance BVH (more than kLinearInstances instances, or PRT_TLAS=1), rebuilt for every prt_set_instances as the
  // reference rebuilds its TLAS every frame (Core/Renderer.cpp:33-41, Core/tiny_bvh.h:1732-1770): the host SAH
  // build + SAH-optimal collapse (bvh_build.h build_tlas8), on the calling thread when the instance set changes,
  // on the worker thread (tlas_worker) in stream order for every later update (ensure_instances)
  bool use_tlas = false;
  int tlas_depth = 0;    // levels the traversal stacks are sized for (>= the current tree's depth)
  int32_t tlas_n = -1;   // instance count of the current tree (-1: none)
  std::unique_ptr<TlasWorker> tlas_worker;
  int32_t tlas_rebuilds = 0, tlas_async = 0;  // since the instance count last changed (diagnostics)
  // pinned staging buffers of ensure_instances' uploads (instance sources, a new tree's nodes / slots / refit order;
  // hipMemcpyAsync from pageable memory may block the host): a buffer is written again only after its copies have
  // run, so the host never waits on queued frames unless it is kStageSlots updates ahead of the GPU
  std::vector<StageSlot> stage;
  uint64_t stage_seq = 0;  // acquisitions so far (StageSlot::seq: the oldest buffer is waited for when all are in use)
  size_t stage_bytes = 0;  // the size the pool was last allocated for
  uint32_t* stage_flag = nullptr;      // one coherent pinned word per staging buffer (64-B stride): TlasJob::flag
  uint32_t* stage_flag_dev = nullptr;  // its device address
  DevBuf spill;  // traversal stack levels beyond the LDS ones (BVHs deeper than 17 levels)
  DevBuf diag;   // SceneDev::diag device counters ([0] traversal stack overflows, cumulative per context)
  // area light (prt_set_area_lights): p0, eu, ev, n, Le, area
  float al[16] = {};
  int32_t area = 0, area_two_sided = 0;
  bool inst_dirty = true;  // the device instance records (k_refit) are out of date
  bool tlas_dirty = true;  // transforms or meshes changed since the instance BVH was last built / refitted
  // sky, lights, camera
  DevBuf sky;
  int32_t skyw = 0, skyh = 0;
  DevBuf srgb;  // 256-entry sRGB -> linear table of the albedo decode
  prt_lights lights{};
  bool have_lights = false;
  prt_camera cam{};
  bool have_camera = false;
  prt_postfx pfx{};  // post-processing off until prt_set_postfx
  DevBuf accprev;    // accumulator before the last frame of a call (screen-pass aberration)
  // accumulation state (Core/Renderer.h:61-63) and scratch
  DevBuf acc, nsamp, dist;
  int32_t accW = 0, accH = 0;
  DevBuf frames, avg, rgb8, counters, hits, tl;
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  // wavefront state of the merged pipeline (frame-in-flight slot 0 and calls in the context stream's order)
  WaveState ws;
  WaveTimers wt = {};
  // the last enqueued render, for its stats (read_stats)
  uint32_t last_iters = 0;
  bool last_timers = false;
  uint64_t last_paths = 0;
  uint64_t carry_segments = 0, carry_shadow = 0;  // ray counts of a call's earlier frame passes
  // sharding (prt_shard_init_rccl / prt_shard_attach_rccl / prt_create_group)
  int32_t sh_kind = 0;  // 0 none, 1 RCCL, 2 local group (this context is member 0)
  int32_t sh_rank = 0, sh_world = 1, sh_tile = 32;
  ncclComm_t comm = nullptr;
  bool own_comm = false;
  std::vector<prt_ctx*> members;  // local group: members 1..world-1, owned by member 0
  DevBuf shtiles, gathered;       // this rank's tile buffer; rank 0: [world][tile buffer] gathered
  hipEvent_t sh_ev = nullptr;     // member: tiles handed to member 0; member 0: untile done
  bool layout_checked = false;    // check_layout_once done
  // frames in flight (prt_set_frames_in_flight): 1 = every call complete in the context stream's order
  int32_t inflight = 1;
  Flight fl[kMaxFlights];
  int32_t next_fl = 0, last_fl = -1;  // the slot of the next call / of the last call still ordering accumulation
  hipEvent_t fl_fork = nullptr;
};

namespace {

// The traversal stacks hold one group per tree level below the root: 8-18 in LDS (by occupancy; 16 in the query
// kernels), deeper levels in HBM spill columns (ensure_spill), up to tinybvh's 64-entry stack (tiny_bvh.h:6315)
constexpr int kMaxBvhDepth = 64;
// tree levels one lane's stack must cover: the deepest BLAS, plus the instance BVH's levels when it is walked
// (its groups sit below the BLAS's: at most one per TLAS level, the last one the remaining instances of a leaf)
int stack_depth(const prt_ctx* c) { return c->max_depth + (c->use_tlas ? c->tlas_depth : 0); }
bool depth_ok(const prt_ctx* c) { return stack_depth(c) <= kMaxBvhDepth; }

// frames in flight: the context stream waits for every call still in flight.  Every entry point but an in-flight
// prt_render starts with it, so its work (and the host waits of drain()) comes after those frames
int join_flights(prt_ctx* c) {
  if (c->last_fl < 0) return PRT_OK;
  HIP_TRY(hipSetDevice(c->device));
  for (Flight& f : c->fl)
    if (f.pending) {
      HIP_TRY(hipStreamWaitEvent(c->stream, f.done, 0));
      f.pending = false;
    }
  c->last_fl = -1;  // the next call's accumulation is ordered through the context stream again
  return PRT_OK;
}

// RCCL calls and waits that involve the peers are bounded (failure detection): a rank whose peers never
// arrive -- at communicator set-up or in a frame's ncclGather -- fails after PRT_RCCL_TIMEOUT_S seconds (default
// 120) with the communicator aborted, instead of hanging in the call or in a later stream wait
double rccl_timeout_s() {
  const char* e = std::getenv("PRT_RCCL_TIMEOUT_S");
  const double v = e ? std::atof(e) : 120.0;
  return v > 0.0 ? v : 120.0;
}
// a non-blocking communicator's call returned ncclInProgress: poll its async state until it settles (bounded)
ncclResult_t rccl_settle(const Rccl* R, ncclComm_t comm, ncclResult_t r) {
  const auto t0 = std::chrono::steady_clock::now();
  const double lim = rccl_timeout_s();
  while (r == ncclInProgress) {
    ncclResult_t st = ncclSuccess;
    if (R->CommGetAsyncError(comm, &st) != ncclSuccess) return ncclSystemError;
    r = st;
    if (r != ncclInProgress) break;
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim) return ncclInProgress;
    std::this_thread::sleep_for(std::chrono::microseconds(200));
  }
  return r;
}
// wait for `s` on an RCCL-sharded context: stream completion, the communicator's async error, or the time limit
// (then the communicator is aborted, which also ends its kernels, and the context cannot shard any more)
int rccl_wait(prt_ctx* c, hipStream_t s, const char* what) {
  const Rccl* R = rccl(nullptr);
  const auto t0 = std::chrono::steady_clock::now();
  const double lim = rccl_timeout_s();
  while (true) {
    const hipError_t e = hipStreamQuery(s);
    if (e == hipSuccess) break;
    if (e != hipErrorNotReady) return fail(PRT_ERR_HIP, std::string(what) + ": " + hipGetErrorString(e));
    ncclResult_t ae = ncclSuccess;
    const bool bad = R && c->comm && R->CommGetAsyncError(c->comm, &ae) == ncclSuccess && ae != ncclSuccess &&
                     ae != ncclInProgress;
    const bool late = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > lim;
    if (bad || late) {
      if (R && c->comm && R->CommAbort) (void)R->CommAbort(c->comm);
      c->comm = nullptr;  // unusable from here on: later sharded frames fail up front
      (void)hipStreamSynchronize(s);  // the aborted collective's kernels end
      return fail(PRT_ERR_HIP, std::string(what) + (bad ? std::string(": RCCL communicator error: ") + R->GetErrorString(ae)
                                                         : ": the RCCL collective did not complete within the time limit "
                                                           "(PRT_RCCL_TIMEOUT_S); communicator aborted"));
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  (void)hipGetLastError();  // hipStreamQuery's hipErrorNotReady
  return PRT_OK;
}

// finish the frames queued on the context stream (and the frames in flight) before a setter overwrites (or frees)
// resident buffers
int drain(prt_ctx* c) {
  const int rc = join_flights(c);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  if (c->sh_kind == 1 && c->comm) return rccl_wait(c, c->stream, "waiting for the context's frames");
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PRT_OK;
}

// triangles per leaf slot the builders may form (binary SAH leaves and the collapse's leaf slots; 2 / 4 measured
// no better on C4)
int max_leaf_tris() { return 3; }

// waves/SIMD of the persistent traversal kernels: the LDS stack (9 / 11 / 14 / 18 groups at 7 / 6 / 5 / 4
// waves) must hold max_depth - 1 groups; deeper BVHs (depth_ok caps them at kMaxBvhDepth = 64 levels) run the
// 4-wave form with HBM spill columns (ensure_spill)
int occ_at(int d) {  // the occupancy a stack of d levels allows (7 waves: re-measured best, profiles/r05_occupancy.txt)
  if (d <= 10) return 7;
  if (d <= 12) return 6;
  if (d <= 15) return 5;
  return 4;
}
int occ_for(const prt_ctx* c) { return occ_at(stack_depth(c)); }

// a pinned staging buffer of at least `bytes` (prt_ctx::stage): a free one (its copies have run), a new one while
// the pool holds fewer than kStageSlots, else the oldest once its copies have run (the only host wait)
int stage_acquire(prt_ctx* c, size_t bytes, StageSlot*& out) {
  StageSlot* pick = nullptr;
  for (StageSlot& t : c->stage) {
    if (t.lost) continue;
    if (t.used) {
      const hipError_t q = hipEventQuery(t.ev);
      if (q == hipErrorNotReady) {
        (void)hipGetLastError();
        continue;
      }
      HIP_TRY(q);
      t.used = false;
    }
    if (!pick || (pick->bytes < bytes && t.bytes >= bytes)) pick = &t;
  }
  if (!pick && c->stage.size() < kStageSlots) {
    c->stage.emplace_back();
    pick = &c->stage.back();
  }
  if (!pick) {  // every buffer in use: wait for the one acquired first
    for (StageSlot& t : c->stage)
      if (!t.lost && (!pick || t.seq < pick->seq)) pick = &t;
    if (!pick) return fail(PRT_ERR_HIP, "no usable staging buffer (earlier updates failed)");
    HIP_TRY(hipEventSynchronize(pick->ev));
    pick->used = false;
  }
  pick->seq = ++c->stage_seq;
  StageSlot& st = *pick;
  if (st.bytes < bytes) {
    if (st.p) HIP_TRY(hipHostFree(st.p));
    st.p = nullptr;
    st.bytes = 0;
    HIP_TRY(hipHostMalloc(&st.p, bytes, hipHostMallocDefault));
    st.bytes = bytes;
  }
  if (!st.ev) HIP_TRY(hipEventCreateWithFlags(&st.ev, hipEventDisableTiming));
  out = &st;
  return PRT_OK;
}
// the copies out of the buffer are enqueued: it is free again once the stream has run them
int stage_release(prt_ctx*, StageSlot& st, hipStream_t s) {
  HIP_TRY(hipEventRecord(st.ev, s));
  st.used = true;
  return PRT_OK;
}

// Instance records on the device (prt_refit.h: MESA inverse, normal matrix, inflated world box): one async copy of
// the transforms + k_refit on the render stream, so frames already queued keep reading the previous instances.
// The instance BVH over those boxes (the same refit_instance on the host) is rebuilt for every update, as the
// reference rebuilds its TLAS every frame (Core/Renderer.cpp:33-41, Core/tiny_bvh.h:1732-1770 BVH::Build over the
// BLASInstances), by the host SAH build + SAH-optimal collapse: on the calling thread when the instance set changes
// (its depth sizes the traversal stacks), and for every later update on the context's worker thread, the render
// stream waiting for that update's build at a host function before its upload (TlasWorker).  The caller only
// copies the update's transforms; every frame walks the tree built over its own instances.
int ensure_instances(prt_ctx* c) {
  if (!c->inst_dirty) return PRT_OK;
  const int32_t n = (int32_t)c->inst_mesh.size();
  const char* te = std::getenv("PRT_TLAS");  // 1: the instance BVH at any instance count (tests)
  const bool use_tlas = n > kLinearInstances || (te && std::atoi(te) == 1);
  // a materials-only update (prt_set_instance_materials) moves no box: the records' kinds are rewritten over
  // unchanged inverses and boxes, and the instance BVH is left as it is
  const bool tree_work = use_tlas && (c->tlas_dirty || !c->use_tlas || c->tlas_n != n);
  const bool async = tree_work && c->use_tlas && c->tlas_n == n && c->tlas_worker;
  if (c->tlas_worker) {
    const TlasWorker::Stats ws = c->tlas_worker->stats();
    if (ws.failed) return fail(PRT_ERR_HIP, "instance BVH build failed on the worker thread: " + ws.err);
  }
  for (int32_t i = 0; i < n; i++)
    if (c->inst_mesh[i] >= c->mesh_host.size()) return fail(PRT_ERR_INVALID_ARGUMENT, "instance references a missing mesh");
  auto fill = [&](InstSrc* src) {  // the refit input of every instance (prt_refit.h)
    for (int32_t i = 0; i < n; i++) {
      InstSrc& s = src[i];
      const uint32_t m = c->inst_mesh[i];
      std::memcpy(s.T, &c->inst_xf[16 * (size_t)i], sizeof(s.T));
      const MeshHost& mh = c->mesh_info[m];
      std::memcpy(s.bmin, mh.bmin, sizeof(s.bmin));
      std::memcpy(s.bmax, mh.bmax, sizeof(s.bmax));
      s.mesh = m;
      s.kind = i < (int32_t)c->inst_kind.size() ? c->inst_kind[i] : 0u;
    }
  };
  // (filled in ordinary memory and copied into the pinned staging buffer in one memcpy: field-by-field stores into
  // pinned memory cost ~10 ms per 10,000 instances on the GPU box, profiles/r06_tlas_drift.txt)
  std::vector<InstSrc>& src = c->inst_stage;
  src.resize(n);
  fill(src.data());
  // the copy of the instance state this update writes: the next one in the ring (frames in flight + 1 copies), once
  // the context stream has waited for the frames that read it
  if (c->isets.size() < (size_t)c->inflight + 1) c->isets.resize((size_t)c->inflight + 1);
  const size_t nx = (c->icur + 1) % c->isets.size();
  InstSet& cur = c->isets[c->icur];
  InstSet& X = c->isets[nx];
  for (size_t k = 0; k < X.nuse; k++) HIP_TRY(hipStreamWaitEvent(c->stream, X.uses[k].second, 0));
  X.nuse = 0;
  // a new instance set: its first tree on the calling thread; the stacks are sized for the largest depth that keeps
  // the traversal's occupancy (and at least the median-split tree's), the cap of the worker's builds
  BuiltTlas8 tree;
  int depth_cap = c->tlas_depth;
  if (tree_work && !async) {
    std::vector<float> boxes(6 * (size_t)n);
    for (int32_t i = 0; i < n; i++) {
      InstDev I;
      refit_instance(src[i], I);
      std::memcpy(&boxes[6 * (size_t)i], I.bmin, 12);
      std::memcpy(&boxes[6 * (size_t)i + 3], I.bmax, 12);
    }
    tree = build_tlas8(boxes.data(), n);
    const int occ = occ_at(c->max_depth + tree.depth);
    depth_cap = std::max(tree.depth, tlas8_median_depth(n));
    while (depth_cap < tree.depth + 4 && occ_at(c->max_depth + depth_cap + 1) == occ &&
           c->max_depth + depth_cap + 1 <= kMaxBvhDepth)
      depth_cap++;
  }
  // buffers sized for n (at least the linear-list size; a tree over n instances has at most max(n, 1) nodes), so
  // later updates never reallocate (a reallocation frees what queued frames read: it drains first, a host wait)
  const size_t cap = (size_t)std::max(n, kLinearInstances);
  const size_t cap_nodes = (size_t)std::max(n, 1);
  if (X.inst.bytes < sizeof(InstDev) * cap || X.inst_src.bytes < sizeof(InstSrc) * cap ||
      (use_tlas && (X.tlas8.bytes < cap_nodes * sizeof(Node8) || X.tlas_slot.bytes < cap_nodes * 32))) {
    const int rc = drain(c);
    if (rc) return rc;
    HIP_TRY(X.inst.ensure(sizeof(InstDev) * cap));
    HIP_TRY(X.inst_src.ensure(sizeof(InstSrc) * cap));
    if (use_tlas) {
      HIP_TRY(X.tlas8.ensure(cap_nodes * sizeof(Node8)));
      HIP_TRY(X.tlas_slot.ensure(cap_nodes * 32));
    }
  }
  // uploads through one pinned staging slot: the instance sources, then the tree's nodes and slots
  const size_t sb_src = sizeof(InstSrc) * (size_t)n;
  const size_t sb_nodes = !tree_work ? 0 : async ? cap_nodes * sizeof(Node8) : tree.nodes.size() * sizeof(Node8);
  const size_t sb_slot = !tree_work ? 0 : async ? cap_nodes * 32 : tree.slot.size() * 4;
  const size_t per = sb_src + (use_tlas ? cap_nodes * (sizeof(Node8) + 32) : 0);
  if (c->stage.size() < kStageSlots || c->stage_bytes < per) {  // the staging buffers this instance set's updates use
    c->stage_bytes = per;
    for (size_t k = c->stage.size(); k < kStageSlots; k++) c->stage.emplace_back();
    if (!c->stage_flag) {
      HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->stage_flag), kStageSlots * 64, hipHostMallocCoherent));
      std::memset(c->stage_flag, 0, kStageSlots * 64);
      HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->stage_flag_dev), c->stage_flag, 0));
    }
    for (StageSlot& t : c->stage) {
      if (t.used && hipEventQuery(t.ev) == hipSuccess) t.used = false;
      (void)hipGetLastError();  // (hipErrorNotReady of a buffer still in use)
      if (!t.used && !t.lost && t.bytes < per) {
        if (t.p) HIP_TRY(hipHostFree(t.p));
        t.p = nullptr;
        t.bytes = 0;
        HIP_TRY(hipHostMalloc(&t.p, per, hipHostMallocDefault));
        t.bytes = per;
      }
    }
  }
  StageSlot* st = nullptr;
  int rc = stage_acquire(c, sb_src + sb_nodes + sb_slot, st);
  if (rc) return rc;
  char* hp = static_cast<char*>(st->p);
  st->lost = true;  // until the copies out of it are enqueued (a failure below leaves it out of the pool)
  std::memcpy(hp, src.data(), sb_src);  // (the worker reads the sources from here)
  HIP_TRY(hipMemcpyAsync(X.inst_src.p, hp, sb_src, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(launch_refit(c->stream, X.inst_src.as<InstSrc>(), n, X.inst.as<InstDev>()));
  if (tree_work) {
    char* q = hp + sb_src;
    if (async) {  // the worker writes the tree into q; the stream's upload waits for it
      const size_t k = (size_t)(st - c->stage.data());  // this buffer's flag word (free with the buffer)
      auto job = std::make_shared<TlasJob>();
      job->src = reinterpret_cast<const InstSrc*>(hp);
      job->n = n;
      job->dst = q;
      job->cap = cap_nodes;
      job->max_depth = c->tlas_depth;
      job->flag = c->stage_flag + 16 * k;
      __atomic_store_n(job->flag, 0u, __ATOMIC_RELAXED);
      HIP_TRY(launch_wait_host(c->stream, c->stage_flag_dev + 16 * k, c->diag.as<uint32_t>() + 2, kHostWaitLimitS));
      c->tlas_worker->submit(job);
    } else {
      std::memcpy(q, tree.nodes.data(), sb_nodes);
      std::memcpy(q + sb_nodes, tree.slot.data(), sb_slot);
    }
    HIP_TRY(hipMemcpyAsync(X.tlas8.p, q, sb_nodes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(X.tlas_slot.p, q + sb_nodes, sb_slot, hipMemcpyHostToDevice, c->stream));
  } else if (use_tlas && &X != &cur) {  // a materials-only update: the current tree, into this copy
    HIP_TRY(hipMemcpyAsync(X.tlas8.p, cur.tlas8.p, cap_nodes * sizeof(Node8), hipMemcpyDeviceToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(X.tlas_slot.p, cur.tlas_slot.p, cap_nodes * 32, hipMemcpyDeviceToDevice, c->stream));
  }
  rc = stage_release(c, *st, c->stream);
  if (rc) return rc;
  st->lost = false;
  c->use_tlas = use_tlas;
  if (!use_tlas) {
    c->tlas_depth = 0;
    c->tlas_n = -1;
  } else if (tree_work && !async) {  // a new instance set
    if (!c->tlas_worker) c->tlas_worker.reset(new TlasWorker());
    c->tlas_worker->seed(tree);
    c->tlas_depth = depth_cap;
    c->tlas_rebuilds = c->tlas_async = 0;
    c->tlas_n = n;
  } else if (async) {
    c->tlas_rebuilds++;
    c->tlas_async++;
  }
  c->icur = nx;
  c->inst_dirty = false;
  c->tlas_dirty = false;
  return PRT_OK;
}

// a frame enqueued on stream st reads the current copy of the instance state: the next update that rewrites it
// waits for this point of st (InstSet)
int record_inst_use(prt_ctx* c, hipStream_t st) {
  InstSet& I = c->isets[c->icur];
  for (size_t k = 0; k < I.nuse; k++)
    if (I.uses[k].first == st) {
      HIP_TRY(hipEventRecord(I.uses[k].second, st));
      return PRT_OK;
    }
  if (I.nuse == I.uses.size()) {
    hipEvent_t e = nullptr;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    I.uses.push_back({st, e});
  }
  I.uses[I.nuse].first = st;
  HIP_TRY(hipEventRecord(I.uses[I.nuse].second, st));
  I.nuse++;
  return PRT_OK;
}

// HBM spill columns for BVHs deeper than the LDS stacks hold (prt_traverse8.h LaneStack): levels beyond the
// query kernels' 16 (the persistent spill form holds 18 in LDS, so this covers it too), one uint2 per level for
// every thread of the launch: `threads` for a query, the persistent spill grid for renders
int ensure_spill(prt_ctx* c, SceneDev& S, size_t threads) {
  const int levels = stack_depth(c) - 1 - kQueryStack;
  S.spill = nullptr;
  S.spill_levels = 0;
  if (levels <= 0) return PRT_OK;
  const size_t need = sizeof(uint2) * (size_t)levels * std::max<size_t>(threads, (size_t)kSpillTraceBlocks * 64u);
  if (c->spill.bytes < need) {
    const int rc = drain(c);
    if (rc) return rc;
    HIP_TRY(c->spill.ensure(need));
  }
  S.spill = c->spill.as<uint2>();
  S.spill_levels = levels;
  return PRT_OK;
}

int scene_ready(prt_ctx* c, SceneDev& S) {
  if (c->mesh_host.empty()) return fail(PRT_ERR_NOT_READY, "no meshes: call prt_set_meshes");
  if (c->inst_mesh.empty()) return fail(PRT_ERR_NOT_READY, "no instances: call prt_set_instances");
  int rc = ensure_instances(c);
  if (rc) return rc;
  std::memset(&S, 0, sizeof(S));
  S.diag = c->diag.as<uint32_t>();
  S.nodes8 = c->nodes8.as<Node8>();
  S.tris = c->tris.as<TriMT>();
  S.stri = c->stri.as<ShadeTri>();
  S.srgb = c->srgb.as<float>();
  S.texels = c->texels.as<uint32_t>();
  S.tex = c->tex.as<TexDev>();
  S.inst = c->isets[c->icur].inst.as<InstDev>();
  S.mesh = c->mesh.as<MeshDev>();
  S.sky = (c->skyw > 0) ? c->sky.as<float>() : nullptr;
  S.ninst = (int32_t)c->inst_mesh.size();
  S.tlas = c->use_tlas ? 1 : 0;
  S.tlas8 = c->use_tlas ? c->isets[c->icur].tlas8.as<Node8>() : nullptr;
  S.tlas_slot = c->use_tlas ? c->isets[c->icur].tlas_slot.as<uint32_t>() : nullptr;
  {  // packed hit word: prim bits for the largest mesh, instance bits above
    uint32_t maxt = 1;
    for (const MeshDev& m : c->mesh_host) maxt = std::max(maxt, m.tri_count);
    uint32_t pb = 1, ib = 0;
    while (pb < 32 && (1ull << pb) < maxt) pb++;
    while ((1ull << ib) < (uint64_t)S.ninst) ib++;
    if (pb + ib > 32) return fail(PRT_ERR_UNSUPPORTED, "mesh size x instance count exceed the 32-bit hit word");
    S.pbits = pb;
  }
  S.skyw = c->skyw;
  S.skyh = c->skyh;
  const prt_lights& L = c->lights;
  std::memcpy(S.ppos, L.point_pos, sizeof(S.ppos));
  std::memcpy(S.pcol, L.point_color, sizeof(S.pcol));
  std::memcpy(S.dpos, L.dir_pos, 12);
  std::memcpy(S.dcol, L.dir_color, 12);
  std::memcpy(S.spos, L.spot_pos, 12);
  std::memcpy(S.scol, L.spot_color, 12);
  std::memcpy(S.srot, L.spot_rot, 12);
  std::memcpy(S.cam, c->cam.pos, 12);
  std::memcpy(S.cam + 3, c->cam.top_left, 12);
  std::memcpy(S.cam + 6, c->cam.top_right, 12);
  std::memcpy(S.cam + 9, c->cam.bottom_left, 12);
  std::memcpy(S.basis, c->cam.right, 12);
  std::memcpy(S.basis + 3, c->cam.up, 12);
  std::memcpy(S.basis + 6, c->cam.ahead, 12);
  S.panini = c->pfx.enabled ? 1 : 0;
  S.pan_d = c->pfx.distortion;
  S.pan_b = panini_scale(c->pfx.fov, c->pfx.distortion);
  std::memcpy(S.al, c->al, sizeof(S.al));
  S.area = c->area;
  S.area_two_sided = c->area_two_sided;
  S.has_diel = 0;
  for (size_t i = 0; i < c->inst_mesh.size() && i < c->inst_kind.size(); i++)
    if (c->inst_kind[i] == kMatDielectric) S.has_diel = 1;
  return PRT_OK;
}

PostDev post_params(const prt_ctx* c, int32_t W, int32_t H) {
  PostDev P{};
  for (int k = 0; k < 4; k++) P.grade[k] = c->pfx.color_grading[k];
  P.vig_int = c->pfx.vignette_intensity;
  P.vig_rad = c->pfx.vignette_radius;
  P.aberration = c->pfx.aberration;
  P.W = W;
  P.H = H;
  return P;
}

int check_params(const prt_render_params* p) {
  if (!p) return fail(PRT_ERR_INVALID_ARGUMENT, "params is NULL");
  if (p->width <= 0 || p->height <= 0 || p->width > 16384 || p->height > 16384)
    return fail(PRT_ERR_INVALID_ARGUMENT, "bad resolution");
  if (p->spp < 0) return fail(PRT_ERR_INVALID_ARGUMENT, "spp < 0");
  if ((p->flags & PRT_FLAG_AA) && (p->spp % 2) != 0)
    return fail(PRT_ERR_INVALID_ARGUMENT, "with PRT_FLAG_AA spp must be even (2 paths per reference frame)");
  if (p->bounces < 0 || p->bounces > 16) return fail(PRT_ERR_INVALID_ARGUMENT, "bounces must be in [0,16]");
  if (p->render_mode < 0 || p->render_mode > 6) return fail(PRT_ERR_INVALID_ARGUMENT, "bad render_mode");
  return PRT_OK;
}

int32_t frames_of(const prt_render_params* p) {
  return (p->flags & PRT_FLAG_AA) ? p->spp / 2 : p->spp;
}

int ensure_state(prt_ctx* c, int32_t W, int32_t H) {
  if (c->accW == W && c->accH == H && c->acc.p) return PRT_OK;
  if (c->acc.p) {  // a new image size: the frames still queued (or in flight) read the old state
    const int rc = drain(c);
    if (rc) return rc;
  }
  const size_t n = (size_t)W * H;
  HIP_TRY(c->acc.ensure(n * 16));
  HIP_TRY(c->nsamp.ensure(n * 4));
  HIP_TRY(c->dist.ensure(n * 4));
  HIP_TRY(hipMemsetAsync(c->acc.p, 0, n * 16, c->stream));
  HIP_TRY(hipMemsetAsync(c->nsamp.p, 0, n * 4, c->stream));
  std::vector<float> d(n, -1.0f);  // Core/Renderer.h:62 (distances = -1 -> first frame resets)
  HIP_TRY(hipMemcpyAsync(c->dist.p, d.data(), n * 4, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  c->accW = W;
  c->accH = H;
  return PRT_OK;
}

// wavefront buffers sized for n items and (bounces-1) (result, throughput) stack levels
// queue counters [iter][path|shadow][kNSub] + traversal fetch counters [iter][path|shadow][8 parts]
constexpr size_t kCtrWords = (size_t)(kMaxIters + 2) * 2 * (kNSub + 8) * kCtrStride;
// shadow-queue entries one shading launch may append per item: <= 4 light-class + 1 area-light ray; the merged
// pipeline (no extensions) shades path 1's last segment and path 2's first in the same launch, 4 + 4
constexpr uint32_t shadow_per_item(bool merge) { return merge ? 8u : 5u; }
int ensure_wave(WaveState& ws, uint32_t n, int bounces, bool ext, bool merge) {
  const uint32_t levels = (uint32_t)std::max(1, bounces - 1);
  // sub-queue t receives the 256-entry chunks c == t (mod kNSub): at most ceil(ceil(n/256)/kNSub) of them
  const uint32_t qcap = 256u * (((n + 255u) / 256u + kNSub - 1) / kNSub);
  if (ws.n >= n && ws.levels >= levels && (ws.ext || !ext) && (ws.merge || !merge) && ws.wave.p) {
    ws.wb.n = n;  // capacity stays; the SoA strides (R/T: depth * n + item) follow the current n
    ws.wb.qcap = qcap;
    ws.wb.scap = shadow_per_item(merge) * qcap;
    ws.wb.merge = merge ? 1 : 0;
    return PRT_OK;
  }
  // merge: two record slots (path 1, path 2) per item for the NEE record, hit point, status and stack
  const size_t ns = merge ? 2ull * n : (size_t)n;
  const size_t qn = (size_t)kNSub * qcap, sn = shadow_per_item(merge) * qn;
  size_t off = 0;
  auto take = [&](size_t bytes) { size_t o = off; off += (bytes + 255) & ~size_t(255); return o; };
  const size_t o_seed = take(4ull * n), o_info = take(4ull * n), o_rinfo = take(4ull * ns), o_ro = take(16ull * n),
               o_rd = take(16ull * n), o_R = take(16ull * ns * levels), o_T = take(16ull * ns * levels),
               o_s1 = take(16ull * n), o_jit = take(8ull * n), o_hit = take(16ull * n), o_ne = take(16ull * ns),
               o_nb = take(16ull * ns), o_nk = take(16ull * ns), o_vis = take(merge ? 8ull * n : 5ull * n),
               o_q0 = take(4 * qn), o_q1 = take(4 * qn), o_shq = take(4 * sn), o_hp = take(16ull * ns),
               o_ctr = take(4 * kCtrWords);
  const size_t o_ro2 = merge ? take(16ull * n) : 0, o_rd2 = merge ? take(16ull * n) : 0,
               o_hit2 = merge ? take(16ull * n) : 0;
  const size_t o_na = ext ? take(16ull * n) : 0, o_dst = ext ? take(4ull * n) : 0,
               o_dro = ext ? take(16ull * n * levels) : 0, o_drd = ext ? take(16ull * n * levels) : 0,
               o_ao = ext ? take(16ull * n) : 0, o_ad = ext ? take(16ull * n) : 0;
  HIP_TRY(ws.wave.ensure(off));
  char* b = ws.wave.as<char>();
  WaveBufs& W = ws.wb;
  W.n = n;
  W.base = 0;
  W.qcap = qcap;
  W.scap = shadow_per_item(merge) * qcap;
  W.seed = (uint32_t*)(b + o_seed); W.info = (uint32_t*)(b + o_info); W.rinfo = (uint32_t*)(b + o_rinfo);
  W.ro = (float4*)(b + o_ro); W.rd = (float4*)(b + o_rd); W.R = (float4*)(b + o_R); W.T = (float4*)(b + o_T);
  W.s1 = (float4*)(b + o_s1); W.jit = (float2*)(b + o_jit); W.hit = (float4*)(b + o_hit);
  W.ne = (float4*)(b + o_ne); W.nb = (float4*)(b + o_nb); W.nk = (float4*)(b + o_nk); W.vis = (uint32_t*)(b + o_vis);
  W.q0 = (uint32_t*)(b + o_q0); W.q1 = (uint32_t*)(b + o_q1); W.shq = (uint32_t*)(b + o_shq); W.hp = (float4*)(b + o_hp);
  W.ctr = (uint32_t*)(b + o_ctr);
  W.na = ext ? (float4*)(b + o_na) : nullptr; W.dst = ext ? (uint32_t*)(b + o_dst) : nullptr;
  W.dro = ext ? (float4*)(b + o_dro) : nullptr; W.drd = ext ? (float4*)(b + o_drd) : nullptr;
  W.ao = ext ? (float4*)(b + o_ao) : nullptr; W.ad = ext ? (float4*)(b + o_ad) : nullptr;
  W.ro2 = merge ? (float4*)(b + o_ro2) : nullptr; W.rd2 = merge ? (float4*)(b + o_rd2) : nullptr;
  W.hit2 = merge ? (float4*)(b + o_hit2) : nullptr;
  W.merge = merge ? 1 : 0;
  ws.n = n;
  ws.levels = levels;
  ws.ext = ext;
  ws.merge = merge;
  return PRT_OK;
}

// the context's running ray totals (prt_ray_totals): bytes 16-31 of the diag buffer, zeroed at prt_create
Counters* ray_totals_dev(prt_ctx* c) { return reinterpret_cast<Counters*>(c->diag.as<char>() + 16); }

// k_shade2 reads its arguments through the kernarg segment (prt_wave2.hip Shade2Args) and flags diag[1] when the
// layout it assumes is not the compiler's (it then shades nothing).  Checked once per context, after its first
// render (one host wait), so stats-less frame loops fail loudly too; prt_ray_totals re-checks it
int check_layout_once(prt_ctx* c, hipStream_t st) {
  if (c->layout_checked) return PRT_OK;
  uint32_t v[2] = {0, 0};
  HIP_TRY(hipMemcpyAsync(v, c->diag.p, 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  if (v[1] != 0) return fail(PRT_ERR_HIP, "k_shade2: kernel-argument layout check failed (Shade2Args)");
  c->layout_checked = true;
  return PRT_OK;
}

// fault injection (tests of the sharded error paths): PRT_FAIL_RENDER=<rank> makes that shard's render fail in
// prepare_render, before anything is enqueued ("all": every context)
int injected_failure(int32_t rank) {
  const char* e = std::getenv("PRT_FAIL_RENDER");
  if (!e || !*e) return PRT_OK;
  if (std::strcmp(e, "all") == 0 || std::atoi(e) == rank)
    return fail(PRT_ERR_HIP, "injected render failure (PRT_FAIL_RENDER) on shard " + std::to_string(rank));
  return PRT_OK;
}

// the wavefront state and frame buffer of a call: slot 0 of the frames in flight and a call in the context stream's
// order share the context's own (they never overlap: the latter joins the flights first)
WaveState& flight_ws(prt_ctx* c, Flight* fl) { return (fl && fl != &c->fl[0]) ? fl->ws : c->ws; }
DevBuf& flight_frames(prt_ctx* c, Flight* fl) { return (fl && fl != &c->fl[0]) ? fl->frames : c->frames; }

// A call's work items (pixels x reference frames) index the shadow-queue entries as 4 x item + k in 29 bits
// (prt_wave2.hip kShIndexMask; the light class takes the top 3), so one pass holds at most 2^27 items
constexpr uint64_t kMaxPassItems = 1ull << 27;

// everything a render needs that can fail: validation and every allocation.  prepare_render enqueues no
// rendering work (ensure_state's first-use clears aside), so a failure leaves the accumulation state as it was
// and a sharded frame can still post its gather (render_sharded)
struct RenderPlan {
  SceneDev S;
  TraceArgs A;
  int32_t F = 0, fmax = 1, npass = 1, F0 = 0;
  uint64_t per = 0;
  bool ext = false, merge = false;
  uint32_t iters = 0;
};

// The merged pipeline (prt_wave2.hip k_shade2m): AA frames of render mode 0 without extensions, in calls small
// enough that their traversal launches are bound by their slowest rays (one launch fewer per frame: world-8 share
// of C4 1.83-1.87 -> 1.74-1.77 ms), not by throughput (the path-2 first segments shaded in partly filled waves
// cost a full C4 frame 1.5 %), up to 2^21 items per call.  PRT_MERGE=0 / 1 forces it off / on (tests).  Its shadow-queue entries index 4 x (slot x n + item) + k in 29 bits: at most 2^26
// items per pass.
constexpr uint64_t kMaxMergedPassItems = 1ull << 26;
bool merge_for(const prt_render_params* p, bool ext, uint64_t per) {
  const bool ok = !ext && p->render_mode == 0 && (p->flags & PRT_FLAG_AA) && p->bounces > 0 && per <= kMaxMergedPassItems;
  const char* e = std::getenv("PRT_MERGE");
  if (e) return ok && std::atoi(e) != 0;
  return ok && per * (uint64_t)frames_of(p) <= (1ull << 21);
}

int prepare_render(prt_ctx* c, const prt_render_params* p, const TileMap& M, int32_t rank, RenderPlan& R,
                   Flight* fl = nullptr) {
  SceneDev& S = R.S;
  int rc = injected_failure(rank);
  if (rc) return rc;
  rc = scene_ready(c, S);
  if (rc) return rc;
  if (!c->have_camera) return fail(PRT_ERR_NOT_READY, "no camera: call prt_set_camera");
  if (!c->have_lights) return fail(PRT_ERR_NOT_READY, "no lights: call prt_set_lights");
  if (!depth_ok(c)) return fail(PRT_ERR_UNSUPPORTED, "BVH deeper than 64 levels");
  // work items are pixels x reference frames (≈ 390 B of wavefront state each); a call holding more than 2^27 of
  // them (≈ 52 GB of state) runs its frames in passes of up to 2^27 items (at least one frame), each folded into
  // the accumulation state in order (the reference's frame sequence).  PRT_MAX_ITEMS sets a smaller pass size
  // (tests run the multi-pass path at small sizes); a frame is never split, so one frame (of this shard) may
  // hold at most 2^27 pixels
  const uint64_t per = (uint64_t)M.items;
  if (per > kMaxPassItems) return fail(PRT_ERR_UNSUPPORTED, "more than 2^27 pixels in one frame of one shard");
  rc = ensure_spill(c, S, 0);
  if (rc) return rc;
  rc = ensure_state(c, p->width, p->height);
  if (rc) return rc;
  const int32_t F = frames_of(p);
  // extensions (area light, dielectric instances) take the EXT instantiations of the shading kernels
  const bool ext = (S.area || S.has_diel) && p->render_mode == 0;
  const bool merge = merge_for(p, ext, per);
  const uint64_t pass_cap = merge ? kMaxMergedPassItems : kMaxPassItems;
  const char* emi = std::getenv("PRT_MAX_ITEMS");
  const uint64_t max_items = emi ? std::min<uint64_t>(std::max<uint64_t>(std::strtoull(emi, nullptr, 10), 1), pass_cap)
                                 : pass_cap;
  const int32_t fmax = (int32_t)std::max<uint64_t>(1, max_items / std::max<uint64_t>(per, 1));
  const int32_t npass = F > fmax ? (F + fmax - 1) / fmax : 1;
  const int32_t F0 = std::min(F, fmax);
  DevBuf& frames = flight_frames(c, fl);
  HIP_TRY(frames.ensure(sizeof(float4) * (size_t)std::max<uint64_t>(per * (uint64_t)F0, 1)));
  TraceArgs& A = R.A;
  A.W = p->width; A.H = p->height; A.bounces = p->bounces; A.flags = p->flags; A.mode = p->render_mode;
  A.frame_index = p->frame_index; A.seed = p->seed; A.frames = F0;
  const uint32_t iters = wave_iters(S.has_diel != 0, p->bounces, p->flags, merge);
  if (iters > (uint32_t)kMaxIters)
    return fail(PRT_ERR_UNSUPPORTED, S.has_diel ? "dielectric path trees exceed the wavefront iteration limit (lower bounces)"
                                                : "too many wavefront iterations");
  // sized for the first (largest) pass; later passes hold no more items
  rc = ensure_wave(flight_ws(c, fl), (uint32_t)(per * (uint64_t)F0), p->bounces, ext, merge);
  if (rc) return rc;
  R.F = F; R.fmax = fmax; R.npass = npass; R.F0 = F0; R.per = per; R.ext = ext; R.merge = merge; R.iters = iters;
  return PRT_OK;
}

// the shared trace + accumulate sequence for prt_render / prt_render_tiles, after prepare_render: enqueues the
// render on the context stream; want_stats: per-launch timers + read_stats() afterwards
// fl: a frame in flight (its stream, wavefront state and frame buffer; the accumulation first waits for acc_after,
// the previous call's last work), else the context stream and state
int enqueue_render_body(prt_ctx* c, const prt_render_params* p, const TileMap& M, RenderPlan& R, float4* avg_dev,
                        uint32_t* rgb8_dev, float4* tiles_dev, bool want_stats, Flight* fl, hipEvent_t acc_after);
// one call's frames on the flight's stream (or the context stream), then the mark of its read of the instance state
int enqueue_render(prt_ctx* c, const prt_render_params* p, const TileMap& M, RenderPlan& R, float4* avg_dev,
                   uint32_t* rgb8_dev, float4* tiles_dev, bool want_stats, Flight* fl = nullptr,
                   hipEvent_t acc_after = nullptr) {
  const int rc = enqueue_render_body(c, p, M, R, avg_dev, rgb8_dev, tiles_dev, want_stats, fl, acc_after);
  const int urc = record_inst_use(c, fl ? fl->stream : c->stream);
  return rc ? rc : urc;
}
int enqueue_render_body(prt_ctx* c, const prt_render_params* p, const TileMap& M, RenderPlan& R, float4* avg_dev,
                        uint32_t* rgb8_dev, float4* tiles_dev, bool want_stats, Flight* fl, hipEvent_t acc_after) {
  SceneDev& S = R.S;
  TraceArgs& A = R.A;
  const int32_t F = R.F, fmax = R.fmax, npass = R.npass;
  const uint64_t per = R.per;
  const bool ext = R.ext;
  const uint32_t iters = R.iters;
  int rc = PRT_OK;
  const hipStream_t st = fl ? fl->stream : c->stream;
  WaveState& ws0 = flight_ws(c, fl);
  LaunchCfg L{st, occ_for(c), 1};
  // frames in flight: from 4 frames in flight on, each chain's wavefront grids are a fraction of the resident blocks,
  // so the chains' persistent traversal launches co-reside instead of taking the whole GPU in turns: a third for
  // calls of up to 2^20 items (C4 world-8 share 1.101-1.109 ms with half grids, 1.055-1.062 with a third, 1.079-1.085
  // with a quarter, 1.32 with an eighth; world 4: 1.940-1.949 / 1.878-1.907 / 1.945-1.953 ms), half above (world 2:
  // 3.56-3.57 ms with half grids, 3.72-3.74 with a quarter) -- profiles/r06_ab_flight_grids.txt
#ifdef PRT_FLIGHT_GW  // (A/B builds only)
  const uint32_t Gw = (fl && c->inflight >= 4) ? (uint32_t)PRT_FLIGHT_GW : 1u;
#else
  const uint32_t Gw = (fl && c->inflight >= 4) ? (per * (uint64_t)R.F0 <= (1ull << 20) ? 3u : 2u) : 1u;
#endif
  const LaunchCfg Lw{st, L.occ, Gw};  // the wavefront chain's launches
  // the call's own events (prt_stats ms / ms_trace) only with stats: each record is a gap between kernels
  if (want_stats) HIP_TRY(hipEventRecord(c->ev[0], st));
  // PRT_TAIL=0 switches the cooperative traversal tail off (prt_persist.h; A/B runs only)
  const char* et = std::getenv("PRT_TAIL");
  const int32_t coop = (et && std::atoi(et) == 0) ? 0 : 1;
  // per-launch traversal timers (HIP events around every k_trace launch) with stats (one-pass calls): each event
  // record costs a few us between kernels, so only the stats calls carry them
  const bool timers = want_stats && npass == 1;
  unsigned long long* tl = nullptr;
  if (want_stats && std::getenv("PRT_DEBUG_QUEUES")) {
    const size_t tlb = 32ull * kTlWaves * (kMaxIters + 2);
    HIP_TRY(c->tl.ensure(tlb));
    HIP_TRY(hipMemsetAsync(c->tl.p, 0, tlb, st));
    tl = c->tl.as<unsigned long long>();
  }
  c->carry_segments = c->carry_shadow = 0;
  const bool post = c->pfx.enabled && !tiles_dev && rgb8_dev && F > 0;
  for (int32_t pass = 0; pass < npass; pass++) {
    const int32_t f0 = pass * fmax, Fb = npass == 1 ? F : std::min(fmax, F - f0);
    const bool last = pass == npass - 1;
    A.frame_index = p->frame_index + f0;
    A.frames = Fb;
    const uint64_t nb = per * (uint64_t)Fb;  // this pass's items
    float4* frames = flight_frames(c, fl).as<float4>();
    rc = ensure_wave(ws0, (uint32_t)nb, p->bounces, ext, R.merge);  // no allocation: prepare_render sized it for pass 0
    if (rc) return rc;
    ws0.wb.base = 0;
    ws0.wb.coop_tail = coop;
    ws0.wb.tl = tl;
    {  // the queue counters and the fetch counters of the iterations this call uses (kMaxIters is the capacity)
      const size_t qw = (size_t)(iters + 2) * 2 * kNSub * kCtrStride;
      const size_t fbase = (size_t)(kMaxIters + 2) * 2 * kNSub * kCtrStride;
      const size_t fw = (size_t)(iters + 2) * 2 * kParts * kCtrStride;
      HIP_TRY(launch_clear2(Lw, ws0.wb.ctr, (uint32_t)qw, ws0.wb.ctr + fbase, (uint32_t)fw));
    }
    if (ext && S.has_diel) HIP_TRY(hipMemsetAsync(ws0.wb.dst, 0, 4ull * ws0.wb.n, st));
    HIP_TRY(launch_wave_init(Lw, S, A, M, ws0.wb, frames));
    for (uint32_t it = 0; it <= iters; it++)
      HIP_TRY(launch_wave2_iter(Lw, S, A, M, ws0.wb, frames, timers ? &c->wt : nullptr, it));
    if (last && want_stats) HIP_TRY(hipEventRecord(c->ev[1], st));
    // post-processing (single-GPU image): the screen pass needs the average and, for the aberration, the
    // accumulator before the last frame
    float4* acc_prev = nullptr;
    if (post && last) {
      const size_t np = (size_t)p->width * p->height;
      if (!avg_dev) { HIP_TRY(c->avg.ensure(np * 16)); avg_dev = c->avg.as<float4>(); }
      if (c->pfx.aberration != 0) { HIP_TRY(c->accprev.ensure(np * 16)); acc_prev = c->accprev.as<float4>(); }
    }
    // frames in flight: the accumulation state (and outputs, ray totals) are updated in call order
    if (acc_after) HIP_TRY(hipStreamWaitEvent(st, acc_after, 0));
    HIP_TRY(launch_accumulate(L, M, Fb, p->flags, frames, c->acc.as<float4>(), c->nsamp.as<int32_t>(),
                              c->dist.as<float>(), avg_dev, post ? nullptr : rgb8_dev, tiles_dev, acc_prev,
                              ws0.wb.ctr, iters, ray_totals_dev(c)));
    if (post && last) {
      // with !accumulates the accumulator held this frame's value until the end-of-frame memset
      const float4* acc_new = (p->flags & PRT_FLAG_ACCUMULATE) ? c->acc.as<float4>() : avg_dev;
      HIP_TRY(launch_postfx(L, post_params(c, p->width, p->height), acc_new, acc_prev, c->nsamp.as<int32_t>(),
                            avg_dev, rgb8_dev));
    }
    if (want_stats && !last) {  // this pass's ray counts, before the next pass clears the counters
      std::vector<uint32_t> ctr((size_t)(iters + 2) * 2 * kNSub * kCtrStride);
      HIP_TRY(hipMemcpyAsync(ctr.data(), ws0.wb.ctr, 4 * ctr.size(), hipMemcpyDeviceToHost, st));
      HIP_TRY(hipStreamSynchronize(st));
      for (uint32_t k = 0; k < iters + 2; k++)  // (+2: the merged path-2 primaries are counted at iters + 1)
        for (uint32_t s2 = 0; s2 < kNSub; s2++) {
          c->carry_segments += ctr[((k * 2 + 0) * kNSub + s2) * kCtrStride];
          c->carry_shadow += ctr[((k * 2 + 1) * kNSub + s2) * kCtrStride];
        }
    }
  }
  if (want_stats) HIP_TRY(hipEventRecord(c->ev[2], st));
  c->last_iters = iters;
  c->last_timers = timers;
  c->last_paths = tile_image_pixels(M) * (uint64_t)F * ((p->flags & PRT_FLAG_AA) ? 2u : 1u);
  return check_layout_once(c, st);
}

// frames in flight: the slot the next call takes (calls with stats or host outputs run in the context stream's
// order instead)
Flight* flight_for(prt_ctx* c, bool sync) {
  return (c->inflight > 1 && !sync && c->sh_kind != 2) ? &c->fl[c->next_fl] : nullptr;
}
// the call of slot f is enqueued: its stream forked from the context stream (fork_flight) before its first work;
// land_flight then joins the call inflight - 1 back into the context stream (its outputs are complete in the
// caller's order from now on), so up to `inflight` calls overlap
int fork_flight(prt_ctx* c, Flight& f) {
  HIP_TRY(hipEventRecord(c->fl_fork, c->stream));
  HIP_TRY(hipStreamWaitEvent(f.stream, c->fl_fork, 0));
  return PRT_OK;
}
int land_flight(prt_ctx* c, Flight& f) {
  HIP_TRY(hipEventRecord(f.done, f.stream));
  const int32_t s = (int32_t)(&f - c->fl), nxt = (s + 1) % c->inflight;
  Flight& o = c->fl[nxt];  // the call inflight - 1 back, whose slot the next call takes
  if (o.pending) {
    HIP_TRY(hipStreamWaitEvent(c->stream, o.done, 0));
    o.pending = false;
  }
  f.pending = true;
  c->last_fl = s;
  c->next_fl = nxt;
  return PRT_OK;
}
// the event the next call's accumulation waits for: the last call still in flight (none: the context stream orders)
hipEvent_t flight_after(const prt_ctx* c) { return c->last_fl >= 0 ? c->fl[c->last_fl].done : nullptr; }

int run_render(prt_ctx* c, const prt_render_params* p, const TileMap& M, float4* avg_dev, uint32_t* rgb8_dev,
               float4* tiles_dev, bool want_stats, int32_t rank = 0, bool sync = true) {
  Flight* f = flight_for(c, want_stats || sync);
  int rc = f ? PRT_OK : join_flights(c);
  if (rc) return rc;
  RenderPlan R;
  rc = prepare_render(c, p, M, rank, R, f);
  if (rc) return rc;
  if (!f) return enqueue_render(c, p, M, R, avg_dev, rgb8_dev, tiles_dev, want_stats);
  rc = fork_flight(c, *f);
  if (rc) return rc;
  rc = enqueue_render(c, p, M, R, avg_dev, rgb8_dev, tiles_dev, false, f, flight_after(c));
  const int lrc = land_flight(c, *f);  // a failed call's partial work joins the context stream too
  if (rc) {
    const std::string why = g_err;
    (void)join_flights(c);
    return fail(rc, why);
  }
  return lrc;
}

// the context's traversal stack overflow count (SceneDev::diag[0]); waits for the context stream.  diag[1] != 0:
// a kernel found its kernarg layout assumption broken (prt_wave2.hip Shade2Args) and did no work; diag[2] != 0: the
// stream's wait for a worker build of the instance BVH timed out (k_wait_host)
uint64_t diag_overflows(prt_ctx* c, bool* layout_ok = nullptr, bool* wait_ok = nullptr) {
  uint32_t v[3] = {0, 0, 0};
  if (hipMemcpyAsync(v, c->diag.p, 12, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
      hipStreamSynchronize(c->stream) != hipSuccess)
    return ~0ull;  // unreadable counts as overflowed: never report a clean run that was not checked
  if (layout_ok) *layout_ok = v[1] == 0;
  if (wait_ok) *wait_ok = v[2] == 0;
  return v[0];
}

// waits for the last render of run_render(..., want_stats = true) and fills its stats
int read_stats(prt_ctx* c, prt_stats* stats) {
#ifdef PRT_LANE_STATS
  HIP_TRY(hipStreamSynchronize(c->stream));
  lane_stats_dump();
#endif
  const uint32_t iters = c->last_iters;
  const bool timers = c->last_timers;
  {
    std::memset(stats, 0, sizeof(*stats));
    // per-launch traversal times summed over every launch
    const bool dump = std::getenv("PRT_DEBUG_QUEUES") != nullptr;
    // the queue counters of the iterations this render used (the whole array with the queue dump)
    std::vector<uint32_t> ctr(dump ? kCtrWords : (size_t)(iters + 2) * 2 * kNSub * kCtrStride);
    HIP_TRY(hipMemcpyAsync(ctr.data(), c->ws.wb.ctr, 4 * ctr.size(), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const WaveTimers& wt = c->wt;
    for (uint32_t k = 0; k <= iters + 1; k++) {  // iteration iters + 1: the merged path-2 primaries (Q2)
      uint64_t qs = 0, qa = 0;
      for (uint32_t s = 0; s < kNSub; s++) {
        qs += ctr[((k * 2 + 0) * kNSub + s) * kCtrStride];
        qa += ctr[((k * 2 + 1) * kNSub + s) * kCtrStride];
      }
      stats->segments += qs;
      stats->shadow_rays += qa;
      float a = 0;
      if (timers && k <= iters) HIP_TRY(hipEventElapsedTime(&a, wt.ev[4 * k + 0], wt.ev[4 * k + 1]));
      stats->ms_closest += a;  // one merged trace launch per iteration plus the final shadow-only one
      if (dump && k < iters)
        std::fprintf(stderr, "prt: iteration %u: %llu closest rays, %llu shadow rays; trace launch %.3f ms\n", k,
                     (unsigned long long)qs, (unsigned long long)qa, a);
    }
    if (dump && c->ws.wb.tl) {  // launch timeline: start -> queue drained -> last wave out (us)
      std::vector<unsigned long long> t(4ull * kTlWaves * (kMaxIters + 2));
      HIP_TRY(hipMemcpy(t.data(), c->tl.p, 8 * t.size(), hipMemcpyDeviceToHost));
      for (uint32_t k = 0; k <= iters; k++) {
        unsigned long long s0 = ~0ull, d0 = ~0ull;
        std::vector<double> ex;
        for (int w = 0; w < kTlWaves; w++) {
          const unsigned long long* r = t.data() + 4 * ((size_t)k * kTlWaves + w);
          if (!r[0]) continue;
          s0 = std::min(s0, r[0]);
          if (r[1]) d0 = std::min(d0, r[1]);
        }
        if (s0 == ~0ull || d0 == ~0ull) continue;
        for (int w = 0; w < kTlWaves; w++) {
          const unsigned long long* r = t.data() + 4 * ((size_t)k * kTlWaves + w);
          if (r[0] && r[2]) ex.push_back(((double)r[2] - (double)d0) / 100.0);
        }
        std::sort(ex.begin(), ex.end());
        auto q = [&](double pp) { return ex.empty() ? 0.0 : ex[std::min(ex.size() - 1, (size_t)(pp * ex.size()))]; };
        std::fprintf(stderr, "prt: trace %u: %zu waves, queue empty after %.1f us; waves out at +%.1f / +%.1f / "
                     "+%.1f / +%.1f us (50/90/99/100 %%)\n", k, ex.size(), (d0 - s0) / 100.0, q(0.5), q(0.9),
                     q(0.99), ex.empty() ? 0.0 : ex.back());
        // diagnostic builds (PRT_TAIL_STATS): where the waves that left last (top 5 %) spent the time after the
        // queue emptied: main loop until their tail entry, then the cooperative tail
        struct Late { double out, entry, tail; unsigned owners, iters; };
        std::vector<Late> late;
        for (int w = 0; w < kTlWaves; w++) {
          const unsigned long long* r = t.data() + 4 * ((size_t)k * kTlWaves + w);
          if (!r[0] || !r[2] || !r[3]) continue;
          unsigned long long e = (r[2] & ~0xFFFFFFFFull) | (r[3] >> 32);
          if (e > r[2]) e -= 1ull << 32;
          late.push_back({((double)r[2] - (double)d0) / 100.0, ((double)e - (double)d0) / 100.0,
                          ((double)r[2] - (double)e) / 100.0, (unsigned)(r[3] & 0xFF),
                          (unsigned)((r[3] >> 8) & 0xFFFFFF)});
        }
        if (!late.empty()) {
          std::sort(late.begin(), late.end(), [](const Late& a, const Late& b) { return a.out < b.out; });
          for (size_t lo : {(size_t)0, late.size() * 95 / 100}) {
            auto med = [&](auto f) {
              std::vector<double> v;
              for (size_t i = lo; i < late.size(); i++) v.push_back(f(late[i]));
              std::sort(v.begin(), v.end());
              return v[v.size() / 2];
            };
            std::fprintf(stderr, "prt:   tail %s: entry +%.1f us after the queue emptied, %.1f us in the tail, %.0f "
                         "owners, %.0f tail iterations (medians over %zu waves)\n", lo ? "last 5%" : "all",
                         med([](const Late& l) { return l.entry; }), med([](const Late& l) { return l.tail; }),
                         med([](const Late& l) { return (double)l.owners; }),
                         med([](const Late& l) { return (double)l.iters; }), late.size() - lo);
          }
        }
      }
    }
    bool layout_ok = true, wait_ok = true;
    stats->stack_overflows = diag_overflows(c, &layout_ok, &wait_ok);
    if (!layout_ok) return fail(PRT_ERR_HIP, "k_shade2: kernel-argument layout check failed (Shade2Args)");
    if (!wait_ok) return fail(PRT_ERR_HIP, "the stream's wait for an instance-BVH build timed out");
    stats->segments += c->carry_segments;  // earlier passes of a call above 2^30 work items
    stats->shadow_rays += c->carry_shadow;
    stats->pipeline = 2;
    stats->iterations = (int32_t)(iters + 1);  // traversal launches
    stats->batches = 1;
    stats->ranks = 1;
    float ms = 0, ms_trace = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[2]));
    HIP_TRY(hipEventElapsedTime(&ms_trace, c->ev[0], c->ev[1]));
    stats->paths = c->last_paths;
    stats->ms = ms;
    stats->ms_trace = ms_trace;
  }
  return PRT_OK;
}

// A rank whose part of a frame failed still posts its part of the frame's ncclGather (zeros), so its peers are
// never left blocked in the collective.  The send buffer is the tile buffer, or (if that could not be allocated)
// any context buffer large enough; root's receive buffer likewise.  With no such buffer the rank aborts its
// communicator: the peers' collective then fails through RCCL instead of completing.
void post_zero_gather(prt_ctx* c, size_t per) {
  const std::string why = g_err;  // the error being reported
  const Rccl* R = rccl(nullptr);
  if (!R || !c->comm) { g_err = why; return; }
  (void)hipSetDevice(c->device);
  (void)hipGetLastError();
  const bool root = c->sh_rank == 0;
  const size_t sb = per * sizeof(float4), rb = (size_t)c->sh_world * sb;
  auto pick = [&](DevBuf& pref, size_t bytes, DevBuf* avoid) -> void* {
    if (pref.bytes >= bytes || pref.ensure(bytes) == hipSuccess) return pref.p;
    for (DevBuf* b : {&c->ws.wave, &c->frames, &c->shtiles, &c->gathered, &c->avg})
      if (b != avoid && b->bytes >= bytes) return b->p;
    return nullptr;
  };
  void* send = pick(c->shtiles, sb, nullptr);
  void* recv = nullptr;
  if (root && send) {
    DevBuf* sendb = nullptr;
    for (DevBuf* b : {&c->shtiles, &c->ws.wave, &c->frames, &c->gathered, &c->avg})
      if (b->p == send) sendb = b;
    recv = pick(c->gathered, rb, sendb);
  }
  if (send && (!root || recv) && hipMemsetAsync(send, 0, sb, c->stream) == hipSuccess) {
    (void)rccl_settle(R, c->comm, R->Gather(send, recv, per * 4, ncclFloat32, 0, c->comm, c->stream));
  } else if (R->CommAbort) {
    (void)R->CommAbort(c->comm);
    c->comm = nullptr;  // unusable from here on: later sharded frames fail up front
  }
  g_err = why;
}

// Sharded frame: every rank renders its tiles into shtiles, rank 0 gathers [world][per] and untiles.
// RCCL: one ncclGather per frame on this rank's stream.  Local group: each member renders on its own stream
// and copies its tile buffer into member 0's gathered buffer (peer copy over xGMI across devices); member 0
// waits for those copies, and the members' next copies wait for member 0's untile.
int render_sharded(prt_ctx* c, const prt_render_params* p, float4* avg_dev, uint32_t* rgb_dev, prt_stats* stats,
                   bool sync) {
  const int32_t W = p->width, H = p->height, ts = c->sh_tile, world = c->sh_world;
  if (c->pfx.enabled && c->pfx.aberration != 0)
    return fail(PRT_ERR_UNSUPPORTED, "chromatic aberration needs the accumulators of neighbouring tiles");
  const TileMap M0 = make_tilemap(W, H, ts, 0, world);
  const size_t per = M0.items;  // tile-buffer elements per rank (rank 0 owns the most)
  std::vector<prt_ctx*> all{c};
  all.insert(all.end(), c->members.begin(), c->members.end());
  const bool root = c->sh_rank == 0;
  const bool coll = c->sh_kind == 1;  // RCCL: the peers of this rank meet it in this frame's ncclGather
  if (coll && !c->comm) return fail(PRT_ERR_HIP, "the RCCL communicator was aborted by an earlier failed frame");
  const Rccl* R = coll ? rccl(nullptr) : nullptr;
  // frames in flight (RCCL shards): the frame's chain, gather and untile on the slot's stream; the accumulation
  // waits for the previous call's untile, so the gathers stay in call order on every rank
  Flight* f = coll ? flight_for(c, stats != nullptr || sync) : nullptr;
  if (!f) {
    const int jrc = join_flights(c);
    if (jrc) return jrc;
  }
  const hipStream_t st = f ? f->stream : c->stream;
  // 1. everything that can fail, on every member, before any render work is enqueued: a failure leaves every
  //    member's accumulation state as it was (the next frame is the one the failed call would have been)
  std::vector<RenderPlan> plans(all.size());
  auto prepare_all = [&]() -> int {
    for (size_t k = 0; k < all.size(); k++) {
      prt_ctx* m = all[k];
      const int32_t rank = c->sh_kind == 2 ? (int32_t)k : c->sh_rank;
      HIP_TRY(hipSetDevice(m->device));
      HIP_TRY(m->shtiles.ensure(per * sizeof(float4)));
      const int rc = prepare_render(m, p, make_tilemap(W, H, ts, rank, world), rank, plans[k], f);
      if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (root) HIP_TRY(c->gathered.ensure((size_t)world * per * sizeof(float4)));
    if (coll && !R) {
      const char* why = "RCCL not loaded";
      (void)rccl(&why);
      return fail(PRT_ERR_UNSUPPORTED, why);
    }
    return PRT_OK;
  };
  // 2. the renders
  auto enqueue_all = [&]() -> int {
    if (f) {
      const int frc = fork_flight(c, *f);
      if (frc) return frc;
    }
    for (size_t k = 0; k < all.size(); k++) {
      prt_ctx* m = all[k];
      const int32_t rank = c->sh_kind == 2 ? (int32_t)k : c->sh_rank;
      HIP_TRY(hipSetDevice(m->device));
      const TileMap M = make_tilemap(W, H, ts, rank, world);
      const hipStream_t ms = f ? st : m->stream;
      if (per > M.items)  // the tail of a shorter rank's buffer (zeros over zeros while a previous gather reads it)
        HIP_TRY(hipMemsetAsync(m->shtiles.as<float4>() + M.items, 0, sizeof(float4) * (per - M.items), ms));
      const int rc = enqueue_render(m, p, M, plans[k], nullptr, nullptr, m->shtiles.as<float4>(), stats != nullptr,
                                    f, f ? flight_after(c) : nullptr);
      if (rc) return rc;
    }
    HIP_TRY(hipSetDevice(c->device));
    return PRT_OK;
  };
  int rc = prepare_all();
  bool forked = false;
  if (!rc) {
    rc = enqueue_all();
    forked = f != nullptr;
  }
  if (rc) {
    // RCCL: the other ranks are already (or soon) inside this frame's ncclGather; post this rank's part (zeros)
    // so they complete, then report the local error (frames in flight: after the earlier calls' gathers)
    const std::string why = g_err;
    if (forked) (void)land_flight(c, *f);
    (void)join_flights(c);
    g_err = why;
    if (coll) post_zero_gather(c, per);
    return rc;
  }
  float4* g = root ? c->gathered.as<float4>() : nullptr;
  if (coll) {
    const ncclResult_t r = rccl_settle(R, c->comm, R->Gather(c->shtiles.p, g, per * 4, ncclFloat32, 0, c->comm, st));
    if (r != ncclSuccess) {
      if (f) (void)land_flight(c, *f);
      return fail(PRT_ERR_HIP, std::string("ncclGather: ") + R->GetErrorString(r));
    }
  } else {
    HIP_TRY(hipMemcpyAsync(g, c->shtiles.p, per * sizeof(float4), hipMemcpyDeviceToDevice, c->stream));
    for (size_t k = 1; k < all.size(); k++) {
      prt_ctx* m = all[k];
      HIP_TRY(hipSetDevice(m->device));
      HIP_TRY(hipStreamWaitEvent(m->stream, c->sh_ev, 0));  // member 0's previous untile read g
      float4* dst = g + k * per;
      if (m->device == c->device)
        HIP_TRY(hipMemcpyAsync(dst, m->shtiles.p, per * sizeof(float4), hipMemcpyDeviceToDevice, m->stream));
      else
        HIP_TRY(hipMemcpyPeerAsync(dst, c->device, m->shtiles.p, m->device, per * sizeof(float4), m->stream));
      HIP_TRY(hipEventRecord(m->sh_ev, m->stream));
    }
    HIP_TRY(hipSetDevice(c->device));
    for (size_t k = 1; k < all.size(); k++) HIP_TRY(hipStreamWaitEvent(c->stream, all[k]->sh_ev, 0));
  }
  if (root && (avg_dev || rgb_dev)) {
    LaunchCfg L{st, occ_for(c)};
    const PostDev P = post_params(c, W, H);
    HIP_TRY(launch_untile(L, W, H, ts, world, (uint32_t)per, g, avg_dev, rgb_dev, c->pfx.enabled ? &P : nullptr));
  }
  if (f) return land_flight(c, *f);
  if (c->sh_ev) HIP_TRY(hipEventRecord(c->sh_ev, c->stream));
  if (stats) {
    prt_stats sum{};
    for (size_t k = 0; k < all.size(); k++) {
      prt_stats st{};
      HIP_TRY(hipSetDevice(all[k]->device));
      int rc = read_stats(all[k], &st);
      if (rc) return rc;
      if (k == 0) sum = st;
      else {
        sum.segments += st.segments;
        sum.shadow_rays += st.shadow_rays;
        sum.paths += st.paths;
        sum.ms = std::max(sum.ms, st.ms);
        sum.ms_trace = std::max(sum.ms_trace, st.ms_trace);
        sum.ms_closest += st.ms_closest;
        sum.stack_overflows = (sum.stack_overflows == ~0ull || st.stack_overflows == ~0ull)
                                  ? ~0ull : sum.stack_overflows + st.stack_overflows;  // ~0: unreadable
      }
    }
    sum.ranks = (int32_t)all.size();
    HIP_TRY(hipSetDevice(c->device));
    if (c->sh_kind == 1) {
      // the gather is part of the frame; a communicator that failed asynchronously (a peer's error, a lost link) or
      // a gather whose peers never arrive is reported within the time limit, not waited on
      const int wrc = rccl_wait(c, c->stream, "sharded frame");
      if (wrc) return wrc;
    }
    *stats = sum;
  }
  return PRT_OK;
}

int shard_setup(prt_ctx* c, int32_t tile) {
  if (tile <= 0 || (tile % 8) != 0) return fail(PRT_ERR_INVALID_ARGUMENT, "tile_size must be a positive multiple of 8");
  c->sh_tile = tile;
  if (!c->sh_ev) HIP_TRY(hipEventCreateWithFlags(&c->sh_ev, hipEventDisableTiming));
  return PRT_OK;
}

// every entry point but an in-flight prt_render first joins the frames in flight (join_flights)
#define PRT_JOIN(ctx)                       \
  do {                                      \
    const int rcj_ = join_flights(ctx);     \
    if (rcj_) return rcj_;                  \
  } while (0)

// a setter of a local group applies to every member (member 0 = the group context itself)
#define PRT_FOR_MEMBERS(call)                 \
  do {                                         \
    for (prt_ctx* m : c->members) {            \
      const int rc_ = (call);                  \
      if (rc_) return rc_;                     \
    }                                          \
  } while (0)

}  // namespace

extern "C" {

int prt_abi_version(void) { return PRT_ABI_VERSION; }
const char* prt_last_error(void) { return g_err.c_str(); }

int prt_device_count(int32_t* count) {
  if (!count) return fail(PRT_ERR_INVALID_ARGUMENT, "count is NULL");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  *count = (e == hipSuccess) ? n : 0;
  return PRT_OK;
}

int prt_create(const prt_device_desc* desc, prt_ctx** out) {
  if (!out) return fail(PRT_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return fail(PRT_ERR_NO_DEVICE, "no HIP device visible");
  const int dev = desc ? desc->device : 0;
  if (dev < 0 || dev >= n) return fail(PRT_ERR_INVALID_ARGUMENT, "device ordinal out of range");
  HIP_TRY(hipSetDevice(dev));
  prt_ctx* c = new prt_ctx();
  c->device = dev;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(PRT_ERR_HIP, "hipStreamCreate failed");
  }
  c->stream = c->own_stream;
  {
    // srgbToLinear of every albedo byte (Scene.cpp:171 on texel/255, BRDF.cpp srgbToLinear); the same
    // float ops and double-precision pow rounded once as the oracle, evaluated on the host
    float lut[256];
    for (int b = 0; b < 256; b++) {
      const float x = (float)b * (1.0f / 255.0f);
      lut[b] = (x <= 0.04045f) ? (x / 12.92f) : (float)std::pow((double)((x + 0.055f) / 1.055f), (double)2.4f);
    }
    if (upload(c->srgb, lut, sizeof(lut)) != hipSuccess) {
      delete c;
      return fail(PRT_ERR_HIP, "srgb table upload failed");
    }
    if (c->diag.ensure(64) != hipSuccess || hipMemset(c->diag.p, 0, 64) != hipSuccess) {
      delete c;
      return fail(PRT_ERR_HIP, "diagnostics buffer allocation failed");
    }
  }
  for (auto& e : c->ev) {
    if (hipEventCreate(&e) != hipSuccess) {
      delete c;
      return fail(PRT_ERR_HIP, "hipEventCreate failed");
    }
  }
  for (auto& e : c->wt.ev) {  // per-launch timers only: no system-scope fence / cache writeback per record
    if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess && hipEventCreate(&e) != hipSuccess) {
      delete c;
      return fail(PRT_ERR_HIP, "hipEventCreate failed");
    }
  }
  *out = c;
  return PRT_OK;
}

int prt_destroy(prt_ctx* c) {
  if (!c) return PRT_OK;
  for (prt_ctx* m : c->members) (void)prt_destroy(m);
  c->members.clear();
  (void)hipSetDevice(c->device);
  (void)join_flights(c);
  if (c->sh_kind == 1 && c->comm) (void)rccl_wait(c, c->stream, "prt_destroy");  // (a stuck gather: aborted)
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (Flight& f : c->fl) {
    if (f.stream) (void)hipStreamSynchronize(f.stream);
    if (f.done) (void)hipEventDestroy(f.done);
    if (f.stream) (void)hipStreamDestroy(f.stream);
  }
  if (c->fl_fork) (void)hipEventDestroy(c->fl_fork);
  if (c->comm && c->own_comm) {
    const Rccl* R = rccl(nullptr);
    if (R) (void)R->CommDestroy(c->comm);
  }
  c->comm = nullptr;
  if (c->sh_ev) (void)hipEventDestroy(c->sh_ev);
  c->tlas_worker.reset();  // every job is done: each one's stream wait ran before the synchronisations above
  for (InstSet& I : c->isets)
    for (auto& u : I.uses) (void)hipEventDestroy(u.second);
  if (c->stage_flag) (void)hipHostFree(c->stage_flag);
  for (StageSlot& st : c->stage) {  // the pinned upload ring (its copies ran: the streams are synchronised)
    if (st.ev) (void)hipEventDestroy(st.ev);
    if (st.p) (void)hipHostFree(st.p);
  }
  for (auto e : c->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto e : c->wt.ev)
    if (e) (void)hipEventDestroy(e);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;  // DevBuf members free their device memory
  return PRT_OK;
}

int prt_set_stream(prt_ctx* c, void* s) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  const int rc = join_flights(c);  // the frames in flight complete in the old stream's order
  if (rc) return rc;
  c->stream = s ? reinterpret_cast<hipStream_t>(s) : c->own_stream;
  return PRT_OK;
}

int prt_set_frames_in_flight(prt_ctx* c, int32_t n) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  if (n < 1 || n > kMaxFlights) return fail(PRT_ERR_INVALID_ARGUMENT, "frames in flight must be 1 to 8");
  if (n > 1 && c->sh_kind == 2) return fail(PRT_ERR_UNSUPPORTED, "frames in flight on a local shard group");
  PRT_JOIN(c);
  HIP_TRY(hipSetDevice(c->device));
  if (n > 1) {
    // only the slots used get a stream: HIP deals a process's streams over its hardware queues (GPU_MAX_HW_QUEUES,
    // 4 by default) as they are created, so streams created and never used would still share queues with the
    // chains that are
    for (int32_t k = 0; k < n; k++) {
      Flight& f = c->fl[k];
      if (!f.stream) HIP_TRY(hipStreamCreateWithFlags(&f.stream, hipStreamNonBlocking));
      if (!f.done) HIP_TRY(hipEventCreateWithFlags(&f.done, hipEventDisableTiming));
    }
    if (!c->fl_fork) HIP_TRY(hipEventCreateWithFlags(&c->fl_fork, hipEventDisableTiming));
  }
  c->inflight = n;
  c->next_fl = 0;
  return PRT_OK;
}

int prt_finish(prt_ctx* c) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  PRT_JOIN(c);
  return PRT_OK;
}

int prt_set_textures(prt_ctx* c, const prt_texture* t, int32_t n) {
  if (!c || (n > 0 && !t) || n < 0) return fail(PRT_ERR_INVALID_ARGUMENT, "bad textures");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  std::vector<uint32_t> all;
  std::vector<TexDev> host(n);
  for (int32_t i = 0; i < n; i++) {
    if (t[i].width <= 0 || t[i].height <= 0 || !t[i].pixels) return fail(PRT_ERR_INVALID_ARGUMENT, "bad texture");
    host[i].offset = (uint32_t)all.size();
    host[i].w = t[i].width;
    host[i].h = t[i].height;
    host[i].pad = 0;
    all.insert(all.end(), t[i].pixels, t[i].pixels + (size_t)t[i].width * t[i].height);
  }
  int rc = drain(c);
  if (rc) return rc;
  HIP_TRY(upload(c->texels, all.data(), all.size() * 4));
  HIP_TRY(upload(c->tex, host.data(), host.size() * sizeof(TexDev)));
  c->tex_host = host;
  PRT_FOR_MEMBERS(prt_set_textures(m, t, n));
  return PRT_OK;
}

int prt_set_meshes(prt_ctx* c, const prt_mesh* m_in, int32_t n) {
  const prt_mesh* m = m_in;
  if (!c || !m || n <= 0) return fail(PRT_ERR_INVALID_ARGUMENT, "bad meshes");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  const int builder = c->builder < 0 ? PRT_BUILDER_HOST_SAH : c->builder;
  const bool gpu = builder == PRT_BUILDER_GPU_LBVH || builder == PRT_BUILDER_GPU_PLOC;
  int rc = drain(c);
  if (rc) return rc;
  const auto t_build0 = std::chrono::steady_clock::now();
  struct GpuMesh { DevBuf nodes, tris; GpuBlasInfo gi; uint32_t node_base, tri_base, prim_base; };
  std::vector<GpuMesh> gm(gpu ? n : 0);
  uint32_t gpu_nodes = 0, gpu_tris = 0;
  std::vector<Node8> nodes8;
  std::vector<TriMT> tris;
  std::vector<ShadeTri> stri;
  std::vector<MeshDev> mh(n);
  std::vector<MeshHost> info(n);
  int maxd = 0;
  for (int32_t i = 0; i < n; i++) {
    const prt_mesh& M = m[i];
    if (M.tri_count <= 0 || M.vertex_count <= 0 || !M.triangles || !M.fixed_normals || !M.fixed_uvs || !M.indices ||
        !M.vertices || !M.face_normals)
      return fail(PRT_ERR_INVALID_ARGUMENT, "mesh " + std::to_string(i) + ": missing arrays");
    const int32_t ntex = (int32_t)c->tex_host.size();
    if (M.albedo_tex < 0 || M.albedo_tex >= ntex)
      return fail(PRT_ERR_INVALID_ARGUMENT, "mesh " + std::to_string(i) + ": albedo texture required (Scene.cpp:160)");
    const int32_t tx[4] = {M.albedo_tex, M.normal_tex, M.metalness_tex, M.emission_tex};
    const TexDev& A = c->tex_host[M.albedo_tex];
    for (int k = 1; k < 4; k++) {
      if (tx[k] >= ntex) return fail(PRT_ERR_INVALID_ARGUMENT, "texture id out of range");
      // every map is indexed with the albedo dimensions (Scene.cpp:79-85,160-165)
      if (tx[k] >= 0 && (c->tex_host[tx[k]].w * (int64_t)c->tex_host[tx[k]].h < (int64_t)A.w * A.h ||
                         c->tex_host[tx[k]].w < A.w))
        return fail(PRT_ERR_INVALID_ARGUMENT, "texture smaller than the albedo map (indexed with albedo dims)");
    }
    for (int64_t k = 0; k < 3 * (int64_t)M.tri_count; k++)
      if (M.indices[k] < 0 || M.indices[k] >= M.vertex_count) return fail(PRT_ERR_INVALID_ARGUMENT, "index out of range");
    const uint32_t tri_base = gpu ? gpu_tris : (uint32_t)tris.size();
    float bmin[3], bmax[3];
    int depth = 0;
    int64_t nnodes = 0, nleaves = 0;
    if (gpu) {  // LBVH or PLOC + SAH-optimal 8-wide collapse on the device (bvh_gpu.hip)
      GpuMesh& g = gm[i];
      DevBuf fat;
      HIP_TRY(upload(fat, M.triangles, 48ull * (size_t)M.tri_count));
      HIP_TRY(g.nodes.ensure(sizeof(Node8) * (size_t)M.tri_count));
      HIP_TRY(g.tris.ensure(sizeof(TriMT) * (size_t)M.tri_count));
      HIP_TRY(gpu_build_blas8(c->stream, fat.as<float>(), M.tri_count, max_leaf_tris(), g.nodes.as<Node8>(), g.tris.as<TriMT>(), &g.gi,
                              builder == PRT_BUILDER_GPU_PLOC));
      fat.release();
      if ((uint64_t)gpu_nodes + g.gi.nodes >= (1ull << 32) || (uint64_t)gpu_tris + g.gi.tris >= (1ull << 32))
        return fail(PRT_ERR_UNSUPPORTED, "too many triangles");
      g.node_base = gpu_nodes;
      g.tri_base = gpu_tris;
      gpu_nodes += g.gi.nodes;
      gpu_tris += g.gi.tris;
      mh[i].root = g.node_base;
      for (int k = 0; k < 3; k++) { bmin[k] = g.gi.bmin[k]; bmax[k] = g.gi.bmax[k]; }
      depth = g.gi.depth; nnodes = g.gi.nodes; nleaves = g.gi.leaves;
    } else {
      // rebase child / triangle offsets into the concatenated arrays
      auto append = [&](BuiltBlas8&& built, std::vector<Node8>& all) -> bool {
        const uint32_t node_base = (uint32_t)all.size();
        if ((uint64_t)tri_base + built.tris.size() >= (1ull << 32) ||
            (uint64_t)node_base + built.nodes.size() >= (1ull << 32))
          return false;
        for (auto& nd : built.nodes) {
          nd.child_base += node_base;
          nd.tri_base += tri_base;
        }
        all.insert(all.end(), built.nodes.begin(), built.nodes.end());
        tris.insert(tris.end(), built.tris.begin(), built.tris.end());
        mh[i].root = node_base;
        std::memcpy(bmin, built.bmin, sizeof(bmin));
        std::memcpy(bmax, built.bmax, sizeof(bmax));
        depth = built.depth; nnodes = (int64_t)built.nodes.size(); nleaves = built.leaves;
        return true;
      };
      const bool ok = append(build_blas8(M.triangles, M.tri_count, max_leaf_tris(), builder == PRT_BUILDER_HOST_SBVH),
                             nodes8);
      if (!ok) return fail(PRT_ERR_UNSUPPORTED, "too many triangles");
    }
    mh[i].prim_base = (uint32_t)stri.size();
    mh[i].vert_base = 0;
    mh[i].tri_count = (uint32_t)M.tri_count;
    for (int k = 0; k < 4; k++) mh[i].tex[k] = tx[k];
    const size_t T = (size_t)M.tri_count;
    for (size_t p = 0; p < T; p++) {
      ShadeTri st;
      std::memset(&st, 0, sizeof(st));
      for (int k = 0; k < 3; k++) {
        const size_t c3 = 3 * p + k;
        const float* vp = M.vertices + 3 * (size_t)M.indices[c3];
        for (int j = 0; j < 3; j++) {
          st.n[3 * k + j] = M.fixed_normals[4 * c3 + j];
          st.p[3 * k + j] = vp[j];
          st.fn[j] = M.face_normals[3 * p + j];
        }
        st.uv[2 * k] = M.fixed_uvs[2 * c3];
        st.uv[2 * k + 1] = M.fixed_uvs[2 * c3 + 1];
      }
      stri.push_back(st);
    }
    // ShadeTri.pad[0]: the primitive's TriMT record (the cooperative traversal tail re-tests a helper's
    // winning triangle from its primitive id, prt_persist.h)
    if (gpu) gm[i].prim_base = mh[i].prim_base;
    else
      for (size_t g = tri_base; g < tris.size(); g++) stri[mh[i].prim_base + tris[g].prim].pad[0] = (uint32_t)g;

    for (int k = 0; k < 3; k++) { info[i].bmin[k] = bmin[k]; info[i].bmax[k] = bmax[k]; }
    info[i].depth = depth;
    info[i].nodes = nnodes;
    info[i].leaves = nleaves;
    info[i].tris = M.tri_count;
    maxd = std::max(maxd, depth);
  }
  c->nodes8.release();
  if (gpu) {  // concatenate the per-mesh device results, rebase offsets, primitive -> triangle records
    HIP_TRY(c->nodes8.ensure(sizeof(Node8) * (size_t)gpu_nodes));
    HIP_TRY(c->tris.ensure(sizeof(TriMT) * (size_t)gpu_tris));
    HIP_TRY(upload(c->stri, stri.data(), stri.size() * sizeof(ShadeTri)));
    for (int32_t i = 0; i < n; i++) {
      GpuMesh& g = gm[i];
      HIP_TRY(hipMemcpyAsync(c->nodes8.as<Node8>() + g.node_base, g.nodes.p, sizeof(Node8) * (size_t)g.gi.nodes,
                             hipMemcpyDeviceToDevice, c->stream));
      HIP_TRY(hipMemcpyAsync(c->tris.as<TriMT>() + g.tri_base, g.tris.p, sizeof(TriMT) * (size_t)g.gi.tris,
                             hipMemcpyDeviceToDevice, c->stream));
      HIP_TRY(gpu_blas_finish(c->stream, c->nodes8.as<Node8>() + g.node_base, g.gi.nodes, g.node_base,
                              c->tris.as<TriMT>() + g.tri_base, g.gi.tris, g.tri_base, c->stri.as<ShadeTri>(),
                              g.prim_base));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    gm.clear();  // the per-mesh device builds were copied into the concatenated arrays
  } else {
    HIP_TRY(upload(c->nodes8, nodes8.data(), nodes8.size() * sizeof(Node8)));
    HIP_TRY(upload(c->tris, tris.data(), tris.size() * sizeof(TriMT)));
    HIP_TRY(upload(c->stri, stri.data(), stri.size() * sizeof(ShadeTri)));
  }
  c->build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_build0).count();
  c->built_with = builder;
  HIP_TRY(upload(c->mesh, mh.data(), mh.size() * sizeof(MeshDev)));
  c->mesh_host = mh;
  c->mesh_info = info;
  c->max_depth = maxd;
  c->inst_dirty = true;
  c->tlas_dirty = true;
  PRT_FOR_MEMBERS(prt_set_meshes(m, m_in, n));
  return PRT_OK;
}

int prt_set_bvh_builder(prt_ctx* c, int32_t builder) {
  if (!c || builder < PRT_BUILDER_HOST_SAH || builder > PRT_BUILDER_GPU_PLOC)
    return fail(PRT_ERR_INVALID_ARGUMENT, "bad BLAS builder");
  c->builder = builder;
  PRT_FOR_MEMBERS(prt_set_bvh_builder(m, builder));
  return PRT_OK;
}

int prt_set_instances(prt_ctx* c, const float* xf, const uint32_t* mi, int32_t n) {
  if (!c || !xf || !mi || n <= 0) return fail(PRT_ERR_INVALID_ARGUMENT, "bad instances");
  // (no join of the frames in flight: the update writes the next copy of the instance state, InstSet)
  if (n > kMaxInstances) return fail(PRT_ERR_UNSUPPORTED, "more than 2^24 instances");
  c->inst_xf.assign(xf, xf + 16 * (size_t)n);
  if ((size_t)n != c->inst_mesh.size()) c->inst_kind.clear();  // materials survive transform updates only
  c->inst_mesh.assign(mi, mi + n);
  c->inst_dirty = true;
  c->tlas_dirty = true;
  HIP_TRY(hipSetDevice(c->device));
  if (!c->mesh_host.empty()) {
    const int rc = ensure_instances(c);
    if (rc) return rc;
  }
  PRT_FOR_MEMBERS(prt_set_instances(m, xf, mi, n));
  return PRT_OK;
}

int prt_set_instance_materials(prt_ctx* c, const int32_t* kinds, int32_t n) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  // (no join of the frames in flight: the update writes the next copy of the instance state, InstSet)
  if (n == 0 || !kinds) {
    c->inst_kind.clear();
  } else {
    if (n != (int32_t)c->inst_mesh.size()) return fail(PRT_ERR_INVALID_ARGUMENT, "one material kind per instance");
    for (int32_t i = 0; i < n; i++)
      if (kinds[i] < PRT_MAT_TEXTURED || kinds[i] > PRT_MAT_MIRROR) return fail(PRT_ERR_INVALID_ARGUMENT, "bad material kind");
    c->inst_kind.assign(kinds, kinds + n);
  }
  c->inst_dirty = true;
  HIP_TRY(hipSetDevice(c->device));
  if (!c->mesh_host.empty() && !c->inst_mesh.empty()) {
    const int rc = ensure_instances(c);
    if (rc) return rc;
  }
  PRT_FOR_MEMBERS(prt_set_instance_materials(m, kinds, n));
  return PRT_OK;
}

int prt_set_area_lights(prt_ctx* c, const prt_area_light* a, int32_t n) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  if (n < 0 || n > 1 || (n == 1 && !a)) return fail(PRT_ERR_UNSUPPORTED, "at most one area light");
  if (n == 0) {
    c->area = 0;
    PRT_FOR_MEMBERS(prt_set_area_lights(m, a, n));
    return PRT_OK;
  }
  const float* u = a->edge_u;
  const float* v = a->edge_v;
  const float cx = u[1] * v[2] - u[2] * v[1], cy = u[2] * v[0] - u[0] * v[2], cz = u[0] * v[1] - u[1] * v[0];
  const float area = sqrtf(cx * cx + cy * cy + cz * cz);
  if (!(area > 0.0f)) return fail(PRT_ERR_INVALID_ARGUMENT, "degenerate area light");
  const float inv = 1.0f / sqrtf(cx * cx + cy * cy + cz * cz);  // normalize(): v * (1 / sqrtf(dot(v, v)))
  const float al[16] = {a->corner[0], a->corner[1], a->corner[2], u[0], u[1], u[2], v[0], v[1], v[2],
                        cx * inv, cy * inv, cz * inv, a->radiance[0], a->radiance[1], a->radiance[2], area};
  std::memcpy(c->al, al, sizeof(al));
  c->area = 1;
  c->area_two_sided = a->two_sided ? 1 : 0;
  PRT_FOR_MEMBERS(prt_set_area_lights(m, a, n));
  return PRT_OK;
}

int prt_set_lights(prt_ctx* c, const prt_lights* l) {
  if (!c || !l) return fail(PRT_ERR_INVALID_ARGUMENT, "bad lights");
  c->lights = *l;
  c->have_lights = true;
  PRT_FOR_MEMBERS(prt_set_lights(m, l));
  return PRT_OK;
}

int prt_set_sky(prt_ctx* c, const float* rgb, int32_t w, int32_t h) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  int rc = drain(c);
  if (rc) return rc;
  if (!rgb || w <= 0 || h <= 0) {
    c->skyw = c->skyh = 0;
    PRT_FOR_MEMBERS(prt_set_sky(m, rgb, w, h));
    return PRT_OK;
  }
  HIP_TRY(upload(c->sky, rgb, (size_t)w * h * 3 * 4));
  c->skyw = w;
  c->skyh = h;
  PRT_FOR_MEMBERS(prt_set_sky(m, rgb, w, h));
  return PRT_OK;
}

int prt_set_camera(prt_ctx* c, const prt_camera* cam) {
  if (!c || !cam) return fail(PRT_ERR_INVALID_ARGUMENT, "bad camera");
  c->cam = *cam;
  c->have_camera = true;
  PRT_FOR_MEMBERS(prt_set_camera(m, cam));
  return PRT_OK;
}

// Camera::Camera (Core/Camera.cpp:29-36): tmpl8 normalize = v * (1/sqrtf(dot))
int prt_camera_look_at(const float pos[3], const float target[3], float aspect, prt_camera* o) {
  if (!pos || !target || !o) return fail(PRT_ERR_INVALID_ARGUMENT, "bad look_at arguments");
  auto nrm = [](V3 v) { return prt::normalize(v); };
  const V3 P = v3(pos[0], pos[1], pos[2]), Tg = v3(target[0], target[1], target[2]);
  const V3 ahead = nrm(Tg - P);
  const V3 right = nrm(cross(ahead, v3(0, 1, 0)));
  const V3 up = nrm(cross(right, ahead));
  const V3 a2 = ahead * 2.0f, ar = aspect * right;
  const V3 TL = P + a2 - ar + up, TR = P + a2 + ar + up, BL = P + a2 - ar - up;
  for (int k = 0; k < 3; k++) o->pos[k] = pos[k];
  o->top_left[0] = TL.x; o->top_left[1] = TL.y; o->top_left[2] = TL.z;
  o->top_right[0] = TR.x; o->top_right[1] = TR.y; o->top_right[2] = TR.z;
  o->bottom_left[0] = BL.x; o->bottom_left[1] = BL.y; o->bottom_left[2] = BL.z;
  o->right[0] = right.x; o->right[1] = right.y; o->right[2] = right.z;
  o->up[0] = up.x; o->up[1] = up.y; o->up[2] = up.z;
  o->ahead[0] = ahead.x; o->ahead[1] = ahead.y; o->ahead[2] = ahead.z;
  return PRT_OK;
}

int prt_postfx_preset(int32_t preset, prt_postfx* o) {
  if (!o || preset < 0 || preset > 1) return fail(PRT_ERR_INVALID_ARGUMENT, "bad post-process preset");
  std::memset(o, 0, sizeof(*o));
  o->enabled = 1;
  if (preset == 0) {  // Camera member defaults (Core/Camera.h:12,23,27): float4{1.f} is all ones
    o->fov = 40.f; o->distortion = 40.f; o->vignette_intensity = 20.f; o->vignette_radius = 0.3f; o->aberration = 0;
    for (int k = 0; k < 4; k++) o->color_grading[k] = 1.f;
  } else {            // P1 (Core/Camera.cpp:18-23, Camera.h:11,20,28); vignetteRadius = vignetteRadius keeps 0.3
    o->fov = 90.f; o->distortion = 2.f; o->vignette_intensity = 5.5f; o->vignette_radius = 0.3f; o->aberration = -1;
    o->color_grading[0] = 1.f; o->color_grading[1] = 1.f; o->color_grading[2] = 1.2f; o->color_grading[3] = 0.f;
  }
  return PRT_OK;
}

int prt_set_postfx(prt_ctx* c, const prt_postfx* pfx) {
  if (!c || !pfx) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx/postfx is NULL");
  c->pfx = *pfx;
  PRT_FOR_MEMBERS(prt_set_postfx(m, pfx));
  return PRT_OK;
}

int prt_reset_accumulation(prt_ctx* c, int32_t full) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  PRT_FOR_MEMBERS(prt_reset_accumulation(m, full));
  if (!c->acc.p) return PRT_OK;
  HIP_TRY(hipSetDevice(c->device));
  const size_t n = (size_t)c->accW * c->accH;
  HIP_TRY(hipMemsetAsync(c->acc.p, 0, n * 16, c->stream));
  if (full) {
    HIP_TRY(hipMemsetAsync(c->nsamp.p, 0, n * 4, c->stream));
    std::vector<float> d(n, -1.0f);
    HIP_TRY(hipMemcpyAsync(c->dist.p, d.data(), n * 4, hipMemcpyHostToDevice, c->stream));
  }
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PRT_OK;
}

// ---- checkpoint / resume of the accumulation state (include/prt.h): header + accumulator (float4) + samples
// (int32) + distances (float), n = accW * accH entries each
namespace {
struct AccHeader {
  char magic[8];
  uint32_t version, header_bytes;
  int32_t w, h, sh_rank, sh_world, sh_tile, sh_kind;
  uint64_t n;
};
constexpr char kAccMagic[8] = {'P', 'R', 'T', 'A', 'C', 'C', 'U', 'M'};
constexpr uint32_t kAccVersion = 1;
uint64_t acc_blob_bytes(uint64_t n) { return sizeof(AccHeader) + n * (16 + 4 + 4); }
}  // namespace

int prt_ray_totals(prt_ctx* c, uint64_t* segments, uint64_t* shadow_rays, int32_t reset) {
  if (!c || !segments || !shadow_rays) return fail(PRT_ERR_INVALID_ARGUMENT, "bad ray totals arguments");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  std::vector<prt_ctx*> all{c};
  all.insert(all.end(), c->members.begin(), c->members.end());
  uint64_t seg = 0, sh = 0;
  for (prt_ctx* m : all) {
    HIP_TRY(hipSetDevice(m->device));
    Counters h{};
    uint32_t dg[3] = {0, 0, 0};
    HIP_TRY(hipMemcpyAsync(&h, ray_totals_dev(m), sizeof(h), hipMemcpyDeviceToHost, m->stream));
    HIP_TRY(hipMemcpyAsync(dg, m->diag.p, 12, hipMemcpyDeviceToHost, m->stream));
    if (reset) HIP_TRY(hipMemsetAsync(ray_totals_dev(m), 0, sizeof(Counters), m->stream));
    HIP_TRY(hipStreamSynchronize(m->stream));
    if (dg[1] != 0) return fail(PRT_ERR_HIP, "k_shade2: kernel-argument layout check failed (Shade2Args)");
    if (dg[2] != 0) return fail(PRT_ERR_HIP, "the stream's wait for an instance-BVH build timed out");
    seg += h.segments;
    sh += h.shadow;
  }
  HIP_TRY(hipSetDevice(c->device));
  *segments = seg;
  *shadow_rays = sh;
  return PRT_OK;
}

int prt_accumulation_bytes(prt_ctx* c, uint64_t* bytes) {
  if (!c || !bytes) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx/bytes is NULL");
  if (!c->members.empty()) return fail(PRT_ERR_UNSUPPORTED, "accumulation checkpoints of a local group");
  *bytes = c->acc.p ? acc_blob_bytes((uint64_t)c->accW * c->accH) : 0;
  return PRT_OK;
}

int prt_save_accumulation(prt_ctx* c, void* blob, uint64_t bytes) {
  if (!c || !blob) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx/blob is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  if (!c->members.empty()) return fail(PRT_ERR_UNSUPPORTED, "accumulation checkpoints of a local group");
  if (!c->acc.p) return fail(PRT_ERR_NOT_READY, "nothing accumulated yet");
  const uint64_t n = (uint64_t)c->accW * c->accH;
  if (bytes < acc_blob_bytes(n)) return fail(PRT_ERR_INVALID_ARGUMENT, "blob smaller than prt_accumulation_bytes");
  AccHeader hd{};
  std::memcpy(hd.magic, kAccMagic, 8);
  hd.version = kAccVersion;
  hd.header_bytes = sizeof(AccHeader);
  hd.w = c->accW;
  hd.h = c->accH;
  hd.sh_rank = c->sh_rank;
  hd.sh_world = c->sh_world;
  hd.sh_tile = c->sh_tile;
  hd.sh_kind = c->sh_kind;
  hd.n = n;
  char* b = static_cast<char*>(blob);
  std::memcpy(b, &hd, sizeof(hd));
  HIP_TRY(hipSetDevice(c->device));
  HIP_TRY(hipMemcpyAsync(b + sizeof(hd), c->acc.p, 16 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(b + sizeof(hd) + 16 * n, c->nsamp.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipMemcpyAsync(b + sizeof(hd) + 20 * n, c->dist.p, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PRT_OK;
}

int prt_load_accumulation(prt_ctx* c, const void* blob, uint64_t bytes) {
  if (!c || !blob) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx/blob is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  if (!c->members.empty()) return fail(PRT_ERR_UNSUPPORTED, "accumulation checkpoints of a local group");
  AccHeader hd{};
  if (bytes < sizeof(hd)) return fail(PRT_ERR_INVALID_ARGUMENT, "truncated accumulation blob");
  std::memcpy(&hd, blob, sizeof(hd));
  if (std::memcmp(hd.magic, kAccMagic, 8) != 0 || hd.version != kAccVersion || hd.header_bytes != sizeof(hd))
    return fail(PRT_ERR_INVALID_ARGUMENT, "not an accumulation blob of this ABI");
  if (hd.w <= 0 || hd.h <= 0 || hd.n != (uint64_t)hd.w * (uint64_t)hd.h || bytes != acc_blob_bytes(hd.n))
    return fail(PRT_ERR_INVALID_ARGUMENT, "accumulation blob size does not match its header");
  if (hd.sh_rank != c->sh_rank || hd.sh_world != c->sh_world || hd.sh_tile != c->sh_tile || hd.sh_kind != c->sh_kind)
    return fail(PRT_ERR_INVALID_ARGUMENT, "accumulation blob of another shard geometry");
  HIP_TRY(hipSetDevice(c->device));
  const int rc = ensure_state(c, hd.w, hd.h);
  if (rc) return rc;
  const char* b = static_cast<const char*>(blob);
  const uint64_t n = hd.n;
  HIP_TRY(hipMemcpyAsync(c->acc.p, b + sizeof(hd), 16 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->nsamp.p, b + sizeof(hd) + 16 * n, 4 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipMemcpyAsync(c->dist.p, b + sizeof(hd) + 20 * n, 4 * n, hipMemcpyHostToDevice, c->stream));
  HIP_TRY(hipStreamSynchronize(c->stream));
  return PRT_OK;
}

int prt_render(prt_ctx* c, const prt_render_params* p, float* avg_rgba, uint32_t* rgb8, uint32_t out_flags,
               prt_stats* stats) {
  if (!c) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx is NULL");
  int rc = check_params(p);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  const size_t np = (size_t)p->width * p->height;
  float4* avg_dev = nullptr;
  uint32_t* rgb_dev = nullptr;
  const bool dev_out = (out_flags & PRT_OUT_DEVICE) != 0;
  const bool root = c->sh_kind == 0 || c->sh_rank == 0;  // the rank whose outputs receive the frame
  if (avg_rgba && root) {
    if (dev_out) avg_dev = reinterpret_cast<float4*>(avg_rgba);
    else { HIP_TRY(c->avg.ensure(np * 16)); avg_dev = c->avg.as<float4>(); }
  }
  if (rgb8 && root) {
    if (dev_out) rgb_dev = rgb8;
    else { HIP_TRY(c->rgb8.ensure(np * 4)); rgb_dev = c->rgb8.as<uint32_t>(); }
  }
  // frames in flight only for device outputs without stats (prt_set_frames_in_flight)
  const bool sync = !dev_out || stats;
  if (c->sh_kind != 0) {
    rc = render_sharded(c, p, avg_dev, rgb_dev, stats, sync);
  } else {
    const TileMap M = make_tilemap(p->width, p->height, 8, 0, 1);
    rc = run_render(c, p, M, avg_dev, rgb_dev, nullptr, stats != nullptr, 0, sync);
    if (!rc && stats) rc = read_stats(c, stats);
  }
  if (rc) return rc;
  if (!dev_out && root) {
    if (avg_rgba) HIP_TRY(hipMemcpyAsync(avg_rgba, avg_dev, np * 16, hipMemcpyDeviceToHost, c->stream));
    if (rgb8) HIP_TRY(hipMemcpyAsync(rgb8, rgb_dev, np * 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
  }
  return PRT_OK;
}

int prt_tile_buffer_pixels(int32_t W, int32_t H, int32_t ts, int32_t world, int64_t* px) {
  if (!px || W <= 0 || H <= 0 || ts <= 0 || (ts % 8) != 0 || world <= 0)
    return fail(PRT_ERR_INVALID_ARGUMENT, "bad tile geometry (tile_size must be a positive multiple of 8)");
  const TileMap M0 = make_tilemap(W, H, ts, 0, world);  // rank 0 owns the most tiles
  *px = (int64_t)M0.items;
  return PRT_OK;
}

int prt_tile_pixel_map(int32_t W, int32_t H, int32_t ts, int32_t rank, int32_t world, int32_t* out) {
  int64_t per = 0;
  int rc = prt_tile_buffer_pixels(W, H, ts, world, &per);
  if (rc) return rc;
  if (!out || rank < 0 || rank >= world) return fail(PRT_ERR_INVALID_ARGUMENT, "bad rank / output");
  const TileMap M = make_tilemap(W, H, ts, rank, world);
  for (int64_t r = 0; r < per; r++) {
    int32_t x = 0, y = 0;
    out[r] = ((uint64_t)r < M.items && item_pixel(M, (uint32_t)r, x, y)) ? y * W + x : -1;
  }
  return PRT_OK;
}

int prt_render_tiles(prt_ctx* c, const prt_render_params* p, int32_t ts, int32_t rank, int32_t world,
                     float* tiles_dev, prt_stats* stats) {
  if (!c || !tiles_dev) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx/tiles is NULL");
    int rc = check_params(p);
  if (rc) return rc;
  if (ts <= 0 || (ts % 8) != 0 || world <= 0 || rank < 0 || rank >= world)
    return fail(PRT_ERR_INVALID_ARGUMENT, "bad tile geometry");
  HIP_TRY(hipSetDevice(c->device));
  const TileMap M = make_tilemap(p->width, p->height, ts, rank, world);
  const TileMap M0 = make_tilemap(p->width, p->height, ts, 0, world);
  if (M0.items > M.items)  // pad the tail of the (equal-size) per-rank buffer
    HIP_TRY(hipMemsetAsync(reinterpret_cast<float4*>(tiles_dev) + M.items, 0, sizeof(float4) * (M0.items - M.items),
                           c->stream));
  // (device tile buffer: a frame in flight unless stats are asked for)
  rc = run_render(c, p, M, nullptr, nullptr, reinterpret_cast<float4*>(tiles_dev), stats != nullptr, rank,
                  stats != nullptr);
  if (!rc && stats) rc = read_stats(c, stats);
  return rc;
}

int prt_untile(prt_ctx* c, const float* gathered, int32_t W, int32_t H, int32_t ts, int32_t world, float* avg_dev,
               uint32_t* rgb8_dev) {
  if (!c || !gathered) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx/gathered is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  int64_t per = 0;
  int rc = prt_tile_buffer_pixels(W, H, ts, world, &per);
  if (rc) return rc;
  HIP_TRY(hipSetDevice(c->device));
  if (c->pfx.enabled && c->pfx.aberration != 0 && rgb8_dev)
    return fail(PRT_ERR_UNSUPPORTED, "chromatic aberration needs the accumulators of neighbouring tiles");
  LaunchCfg L{c->stream, occ_for(c)};
  const PostDev P = post_params(c, W, H);
  HIP_TRY(launch_untile(L, W, H, ts, world, (uint32_t)per, reinterpret_cast<const float4*>(gathered),
                        reinterpret_cast<float4*>(avg_dev), rgb8_dev, c->pfx.enabled ? &P : nullptr));
  return PRT_OK;
}

int prt_trace_primary(prt_ctx* c, int32_t W, int32_t H, prt_hit* hits, uint32_t out_flags, prt_stats* stats) {
  if (!c || !hits || W <= 0 || H <= 0) return fail(PRT_ERR_INVALID_ARGUMENT, "bad arguments");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  HIP_TRY(hipSetDevice(c->device));
  SceneDev S;
  int rc = scene_ready(c, S);
  if (rc) return rc;
  if (!c->have_camera) return fail(PRT_ERR_NOT_READY, "no camera");
  if (!depth_ok(c)) return fail(PRT_ERR_UNSUPPORTED, "BVH deeper than 64 levels");
  const TileMap M = make_tilemap(W, H, 8, 0, 1);
  const size_t n = (size_t)W * H;
  rc = ensure_spill(c, S, (size_t)M.items + 256);
  if (rc) return rc;
  HitOut* out = reinterpret_cast<HitOut*>(hits);
  const bool dev_out = (out_flags & PRT_OUT_DEVICE) != 0;
  if (!dev_out) { HIP_TRY(c->hits.ensure(n * sizeof(HitOut))); out = c->hits.as<HitOut>(); }
  HIP_TRY(c->counters.ensure(sizeof(Counters)));
  HIP_TRY(hipMemsetAsync(c->counters.p, 0, sizeof(Counters), c->stream));
  LaunchCfg L{c->stream, occ_for(c)};
  HIP_TRY(hipEventRecord(c->ev[0], c->stream));
  HIP_TRY(launch_primary_hits(L, S, M, out, c->counters.as<Counters>()));
  HIP_TRY(hipEventRecord(c->ev[2], c->stream));
  if (!dev_out) HIP_TRY(hipMemcpyAsync(hits, out, n * sizeof(HitOut), hipMemcpyDeviceToHost, c->stream));
  if (stats || !dev_out) HIP_TRY(hipStreamSynchronize(c->stream));
  if (stats) {
    Counters h{};
    HIP_TRY(hipMemcpy(&h, c->counters.p, sizeof(h), hipMemcpyDeviceToHost));
    float ms = 0;
    HIP_TRY(hipEventElapsedTime(&ms, c->ev[0], c->ev[2]));
    std::memset(stats, 0, sizeof(*stats));
    stats->ms_closest = ms;
    stats->segments = h.segments;
    stats->shadow_rays = 0;
    stats->paths = n;
    stats->ms = ms;
    stats->ms_trace = ms;
    stats->stack_overflows = diag_overflows(c);
  }
  return PRT_OK;
}

static int ray_query(prt_ctx* c, int32_t n, const float* O, const float* D, const float* tmax, void* out, bool any) {
  if (!c || n < 0 || (n > 0 && (!O || !D || !out)) || (any && n > 0 && !tmax))
    return fail(PRT_ERR_INVALID_ARGUMENT, "bad ray query arguments");
  PRT_JOIN(c);
  if (n == 0) return PRT_OK;
  HIP_TRY(hipSetDevice(c->device));
  SceneDev S;
  int rc = scene_ready(c, S);
  if (rc) return rc;
  if (!depth_ok(c)) return fail(PRT_ERR_UNSUPPORTED, "BVH deeper than 64 levels");
  rc = ensure_spill(c, S, (size_t)n + 256);
  if (rc) return rc;
  DevBuf dO, dD, dT, dOut;
  auto cleanup = [&]() { dO.release(); dD.release(); dT.release(); dOut.release(); };
  const size_t outb = (size_t)n * (any ? 4 : sizeof(HitOut));
  if (upload(dO, O, (size_t)n * 12) != hipSuccess || upload(dD, D, (size_t)n * 12) != hipSuccess ||
      (tmax && upload(dT, tmax, (size_t)n * 4) != hipSuccess) || dOut.ensure(outb) != hipSuccess) {
    cleanup();
    return fail(PRT_ERR_OUT_OF_MEMORY, "ray buffers");
  }
  LaunchCfg L{c->stream, occ_for(c)};
  hipError_t e = any ? launch_occluded(L, S, n, dO.as<float>(), dD.as<float>(), dT.as<float>(), dOut.as<int32_t>())
                     : launch_intersect(L, S, n, dO.as<float>(), dD.as<float>(), tmax ? dT.as<float>() : nullptr,
                                        dOut.as<HitOut>());
  if (e == hipSuccess) e = hipMemcpyAsync(out, dOut.p, outb, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  cleanup();
  if (e != hipSuccess) return fail(PRT_ERR_HIP, std::string("ray query: ") + hipGetErrorString(e));
  return PRT_OK;
}

int prt_intersect(prt_ctx* c, int32_t n, const float* O, const float* D, const float* tmax, prt_hit* hits) {
  return ray_query(c, n, O, D, tmax, hits, false);
}
int prt_occluded(prt_ctx* c, int32_t n, const float* O, const float* D, const float* tmax, int32_t* occ) {
  return ray_query(c, n, O, D, tmax, occ, true);
}

int prt_brdf_probe(prt_ctx* c, int32_t op, int32_t n, const float* in, float* out) {
  if (!c || n < 0 || (n > 0 && (!in || !out)) || op < PRT_PROBE_EVAL || op > PRT_PROBE_VNDF)
    return fail(PRT_ERR_INVALID_ARGUMENT, "bad BRDF probe arguments");
  if (n == 0) return PRT_OK;
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  HIP_TRY(hipSetDevice(c->device));
  DevBuf din, dout;
  HIP_TRY(upload(din, in, 24ull * 4 * (size_t)n));
  HIP_TRY(dout.ensure(8ull * 4 * (size_t)n));
  hipError_t e = launch_brdf_probe(c->stream, op, n, din.as<float>(), dout.as<float>());
  if (e == hipSuccess) e = hipMemcpyAsync(out, dout.p, 8ull * 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return fail(PRT_ERR_HIP, std::string("BRDF probe: ") + hipGetErrorString(e));
  return PRT_OK;
}

int prt_shard_unique_id(uint8_t id[PRT_SHARD_ID_BYTES]) {
  if (!id) return fail(PRT_ERR_INVALID_ARGUMENT, "id is NULL");
  static_assert(sizeof(ncclUniqueId) == PRT_SHARD_ID_BYTES, "ncclUniqueId size");
  const char* why = nullptr;
  const Rccl* R = rccl(&why);
  if (!R) return fail(PRT_ERR_UNSUPPORTED, why);
  ncclUniqueId u;
  const ncclResult_t r = R->GetUniqueId(&u);
  if (r != ncclSuccess) return fail(PRT_ERR_HIP, std::string("ncclGetUniqueId: ") + R->GetErrorString(r));
  std::memcpy(id, &u, sizeof(u));
  return PRT_OK;
}

int prt_shard_init_rccl(prt_ctx* c, const uint8_t id[PRT_SHARD_ID_BYTES], int32_t rank, int32_t world, int32_t tile) {
  if (!c || !id || world <= 0 || rank < 0 || rank >= world) return fail(PRT_ERR_INVALID_ARGUMENT, "bad shard rank / world");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  if (c->sh_kind != 0) return fail(PRT_ERR_INVALID_ARGUMENT, "context is already sharded");
  int rc = shard_setup(c, tile);
  if (rc) return rc;
  const char* why = nullptr;
  const Rccl* R = rccl(&why);
  if (!R) return fail(PRT_ERR_UNSUPPORTED, why);
  HIP_TRY(hipSetDevice(c->device));
  ncclUniqueId u;
  std::memcpy(&u, id, sizeof(u));
  ncclComm_t comm = nullptr;
  ncclResult_t r;
  if (R->CommInitRankConfig) {  // non-blocking set-up, polled: ranks that never join make it fail, not hang
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    r = R->CommInitRankConfig(&comm, world, u, rank, &cfg);
    if (comm && (r == ncclSuccess || r == ncclInProgress)) r = rccl_settle(R, comm, r);
    if (r == ncclInProgress) {
      if (R->CommAbort) (void)R->CommAbort(comm);
      return fail(PRT_ERR_HIP, "ncclCommInitRank: the other ranks did not join within the time limit (PRT_RCCL_TIMEOUT_S)");
    }
    if (r != ncclSuccess && comm && R->CommAbort) (void)R->CommAbort(comm);
  } else {
    r = R->CommInitRank(&comm, world, u, rank);
  }
  if (r != ncclSuccess) return fail(PRT_ERR_HIP, std::string("ncclCommInitRank: ") + R->GetErrorString(r));
  c->comm = comm;
  c->own_comm = true;
  c->sh_kind = 1;
  c->sh_rank = rank;
  c->sh_world = world;
  return PRT_OK;
}

int prt_shard_attach_rccl(prt_ctx* c, void* comm, int32_t tile) {
  if (!c || !comm) return fail(PRT_ERR_INVALID_ARGUMENT, "ctx / comm is NULL");
  PRT_JOIN(c);  // frames in flight complete first (prt_set_frames_in_flight)
  if (c->sh_kind != 0) return fail(PRT_ERR_INVALID_ARGUMENT, "context is already sharded");
  int rc = shard_setup(c, tile);
  if (rc) return rc;
  const char* why = nullptr;
  const Rccl* R = rccl(&why);
  if (!R) return fail(PRT_ERR_UNSUPPORTED, why);
  ncclComm_t cm = reinterpret_cast<ncclComm_t>(comm);
  int n = 0, r = 0;
  if (R->CommCount(cm, &n) != ncclSuccess || R->CommUserRank(cm, &r) != ncclSuccess)
    return fail(PRT_ERR_INVALID_ARGUMENT, "not a usable ncclComm_t");
  c->comm = cm;
  c->own_comm = false;
  c->sh_kind = 1;
  c->sh_rank = r;
  c->sh_world = n;
  return PRT_OK;
}

int prt_create_group(const prt_device_desc* devs, int32_t n, int32_t tile, prt_ctx** out) {
  if (!out) return fail(PRT_ERR_INVALID_ARGUMENT, "out is NULL");
  *out = nullptr;
  if (!devs || n <= 0 || n > 64) return fail(PRT_ERR_INVALID_ARGUMENT, "1..64 devices");
  prt_ctx* g = nullptr;
  int rc = prt_create(&devs[0], &g);
  if (rc) return rc;
  rc = shard_setup(g, tile);
  for (int32_t k = 1; k < n && !rc; k++) {
    prt_ctx* m = nullptr;
    rc = prt_create(&devs[k], &m);
    if (!rc) {
      g->members.push_back(m);
      rc = shard_setup(m, tile);
    }
  }
  if (!rc) {  // peer access between distinct devices (the tile copies go device to device)
    for (prt_ctx* m : g->members) {
      if (m->device == g->device) continue;
      (void)hipSetDevice(m->device);
      const hipError_t e = hipDeviceEnablePeerAccess(g->device, 0);
      if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
    }
    (void)hipSetDevice(g->device);
  }
  if (rc) {
    const std::string msg = g_err;
    (void)prt_destroy(g);
    return fail(rc, msg);
  }
  g->sh_kind = 2;
  g->sh_rank = 0;
  g->sh_world = n;
  *out = g;
  return PRT_OK;
}

int prt_get_shard_info(prt_ctx* c, prt_shard_info* info) {
  if (!c || !info) return fail(PRT_ERR_INVALID_ARGUMENT, "bad arguments");
  info->rank = c->sh_rank;
  info->world = c->sh_world;
  info->tile_size = c->sh_tile;
  info->transport = c->sh_kind;
  return PRT_OK;
}

int prt_get_scene_info(prt_ctx* c, prt_scene_info* info) {
  if (!c || !info) return fail(PRT_ERR_INVALID_ARGUMENT, "bad arguments");
  std::memset(info, 0, sizeof(*info));
  for (const MeshHost& m : c->mesh_info) {
    info->blas_nodes += m.nodes;
    info->blas_leaves += m.leaves;
    info->triangles += m.tris;
  }
  info->max_depth = c->max_depth;
  info->tlas_depth = c->use_tlas ? c->tlas_depth : 0;
  info->tlas_rebuilds = c->tlas_rebuilds;
  info->tlas_async = c->tlas_async;
  info->tlas_median = 0;
  info->tlas_build_ms = info->tlas_build_cpu_ms = 0.0f;
  if (c->tlas_worker) {
    const TlasWorker::Stats ws = c->tlas_worker->stats();
    info->tlas_median = ws.median;
    info->tlas_build_ms = (float)ws.ms;
    info->tlas_build_cpu_ms = (float)ws.cpu_ms;
  }
  info->build_ms = c->build_ms;
  info->builder = c->built_with;
  size_t ib = 0;
  for (const InstSet& I : c->isets) ib += I.inst.bytes + I.inst_src.bytes + I.tlas8.bytes + I.tlas_slot.bytes;
  info->device_bytes = (int64_t)(c->nodes8.bytes + c->tris.bytes + c->stri.bytes + c->texels.bytes + c->sky.bytes + ib);
  return PRT_OK;
}

}  // extern "C"
