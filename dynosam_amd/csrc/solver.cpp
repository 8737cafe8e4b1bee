// solver.cpp — dynohip C-ABI: handle, device buffers, GTSAM 4.2.0
// Levenberg–Marquardt control loop driving the HIP kernels.
//
// Replaces `gtsam::LevenbergMarquardtOptimizer(graph, values,
// LevenbergMarquardtParams()).optimize()` at RGBDBackendModule.cc:207-231
// and :364-383. LM semantics: SURVEY.md Appendix A (GTSAM 4.2.0
// LevenbergMarquardtOptimizer::tryLambda / iterate, NonlinearOptimizer::
// defaultOptimize, checkConvergence). Only ~3 scalars cross to the host per
// inner iteration.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <string>
#include <memory>
#include <vector>

#include "../../include/dynohip.h"
#include "kernels.hpp"
#include "plan.hpp"
#include "prepared.hpp"
#include "plan_pool.hpp"

using namespace dynohip;

namespace {

// Process-wide cache of device allocations, per device. A destroyed handle
// (or a buffer that grows) gives its allocations back here instead of calling
// hipFree (a device-wide synchronising call, ~0.2 ms each, 12 ms for a whole
// C2 handle), and the next allocation of a similar size takes one back: the
// reference constructs a fresh LevenbergMarquardtOptimizer per call
// (RGBDBackendModule.cc:207,364), and a fresh handle per call then costs no
// device allocation at all after the first. Held bytes are capped at
// DYNOHIP_POOL_MAX_MB (default 16384) and a quarter of the device's memory;
// dynohip_pool_trim() frees them, and an allocation that fails for lack of
// memory frees its device's cached blocks and tries again.
class DevPool {
 public:
  static DevPool& get() {
    static DevPool* p = new DevPool();   // never destroyed (process exit releases the device)
    return *p;
  }
  // a cached block of `bytes` <= size <= 2 * bytes on `dev`, or nullptr
  void* take(int dev, size_t bytes, size_t* got) {
    std::lock_guard<std::mutex> lk(mu_);
    size_t best = SIZE_MAX;
    size_t bi = 0;
    for (size_t i = 0; i < free_.size(); ++i) {
      const Blk& b = free_[i];
      if (b.dev == dev && b.bytes >= bytes && b.bytes <= 2 * bytes + 4096 && b.bytes < best) {
        best = b.bytes;
        bi = i;
      }
    }
    if (best == SIZE_MAX) return nullptr;
    void* p = free_[bi].p;
    *got = free_[bi].bytes;
    held_ -= free_[bi].bytes;
    free_[bi] = free_.back();
    free_.pop_back();
    return p;
  }
  void give(int dev, void* p, size_t bytes) {
    if (!p) return;
    size_t total = 0;   // the cache keeps at most a quarter of the device's memory
    if (hipDeviceTotalMem(&total, dev) != hipSuccess) total = 0;
    const size_t limit = total ? std::min(max_bytes_, total / 4) : max_bytes_;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (held_ + bytes <= limit) {
        free_.push_back({p, bytes, dev});
        held_ += bytes;
        return;
      }
    }
    (void)hipFree(p);
  }
  // frees the cached blocks of `dev` (all devices for dev < 0)
  size_t trim(int dev = -1) {
    std::vector<Blk> all;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (dev < 0) {
        all.swap(free_);
        held_ = 0;
      } else {
        for (size_t i = 0; i < free_.size();)
          if (free_[i].dev == dev) {
            all.push_back(free_[i]);
            held_ -= free_[i].bytes;
            free_[i] = free_.back();
            free_.pop_back();
          } else {
            ++i;
          }
      }
    }
    size_t n = 0;
    int cur = 0;
    (void)hipGetDevice(&cur);
    for (const Blk& b : all) {
      (void)hipSetDevice(b.dev);
      (void)hipFree(b.p);
      n += b.bytes;
    }
    (void)hipSetDevice(cur);
    return n;
  }

 private:
  DevPool() {
    const char* e = std::getenv("DYNOHIP_POOL_MAX_MB");
    max_bytes_ = (e ? std::strtoull(e, nullptr, 10) : 16384ull) << 20;
  }
  struct Blk {
    void* p;
    size_t bytes;
    int dev;
  };
  std::mutex mu_;
  std::vector<Blk> free_;
  size_t held_ = 0, max_bytes_ = 0;
};

// Device buffer that keeps its allocation: a handle re-planned for another
// graph (the next sliding window, the next full-batch call) reuses it when it
// is large enough; otherwise, and when the handle is destroyed, the
// allocation goes back to the process-wide DevPool. Contents are not
// preserved across alloc().
template <typename T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  size_t cap = 0;
  int dev = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;              // one owner per allocation
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  // exchange allocations with another buffer (the LM's accepted step swaps
  // current and candidate values): every field, since pooled blocks of one
  // count can differ in capacity
  void swap(DevBuf& o) {
    std::swap(p, o.p);
    std::swap(n, o.n);
    std::swap(cap, o.cap);
    std::swap(dev, o.dev);
  }
  // The block goes to the pool, where another handle (another thread, another
  // stream) may take it at once: it is released only while the owning
  // handle's stream is idle. Every path that can grow a buffer runs after a
  // stream synchronisation (dynohip_set_values before re-planning,
  // dynohip_values_snapshot, dynohip_destroy), and no buffer is grown twice
  // between two synchronisations.
  void release() {
    if (p) DevPool::get().give(dev, p, cap * sizeof(T));
    p = nullptr;
    n = cap = 0;
  }
  hipError_t alloc(size_t count) {
    if (count <= cap) {
      n = count;
      return hipSuccess;
    }
    release();
    (void)hipGetDevice(&dev);
    const size_t c = count + count / 8;   // some headroom for the next graph
    size_t got = 0;
    if (void* q = DevPool::get().take(dev, count * sizeof(T), &got)) {
      p = static_cast<T*>(q);
      n = count;
      cap = got / sizeof(T);
      return hipSuccess;
    }
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p), c * sizeof(T));
    if (e == hipErrorOutOfMemory) {
      // blocks too small for this request may sit in the cache: give this
      // device's back and try once more (without the headroom)
      (void)hipGetLastError();
      DevPool::get().trim(dev);
      e = hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T));
      if (e == hipSuccess) {
        n = cap = count;
        return hipSuccess;
      }
    }
    if (e != hipSuccess) {
      p = nullptr;
      return e;
    }
    n = count;
    cap = c;
    return hipSuccess;
  }
  template <class Alloc>
  hipError_t upload(const std::vector<T, Alloc>& v, hipStream_t s) {
    hipError_t e = alloc(v.size());
    if (e != hipSuccess || v.empty()) return e;
    return hipMemcpyAsync(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s);
  }
};

// Streams, events and the pinned result buffer of a handle, recycled the
// same way (creating them cost ~5 ms per handle).
struct HandleRes {
  int device = 0;
  hipStream_t stream = nullptr, side = nullptr;
  hipEvent_t ev_main = nullptr, ev_side = nullptr, ev_res = nullptr;
  hipEvent_t ev[9] = {};
  double* hres = nullptr;
  char* stage[2] = {nullptr, nullptr};   // pinned upload staging: early (factor records), rest
  size_t stage_cap[2] = {0, 0};
};

class ResPool {
 public:
  static ResPool& get() {
    static ResPool* p = new ResPool();
    return *p;
  }
  bool take(int dev, HandleRes* out) {
    std::lock_guard<std::mutex> lk(mu_);
    for (size_t i = 0; i < free_.size(); ++i)
      if (free_[i].device == dev) {
        *out = free_[i];
        free_[i] = free_.back();
        free_.pop_back();
        return true;
      }
    return false;
  }
  void give(const HandleRes& r) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.push_back(r);
  }

 private:
  std::mutex mu_;
  std::vector<HandleRes> free_;
};

// A plan's host arrays go to the device through pinned staging buffers of
// the handle (recycled with its streams): packed into the buffer, each
// array then one asynchronous DMA. From pageable memory the runtime stages
// every array itself, one copy at a time on the calling thread.
struct Uploads {
  struct Item {
    void* dev;
    const void* host;
    size_t bytes, off;
  };
  std::vector<Item> items;
  size_t total = 0;
  // (v is read at run(): it must outlive the call)
  template <typename T, class Alloc>
  hipError_t add(DevBuf<T>& d, const std::vector<T, Alloc>& v) {
    const hipError_t e = d.alloc(v.size());
    if (e != hipSuccess || v.empty()) return e;
    items.push_back({d.p, v.data(), v.size() * sizeof(T), total});
    total += (v.size() * sizeof(T) + 255) & ~size_t{255};
    return hipSuccess;
  }
  // Packs a chunk table and the arrays into `buf` (pinned, grown to fit), on
  // the planner's workers or on this thread, copies it to `dstage` in one
  // transfer and places the pieces with one kernel (instead of one DMA per
  // array: ~50 per plan, each a few microseconds of GPU time), all on `st`
  // without waiting: the caller synchronises before the buffers are reused.
  hipError_t run(char*& buf, size_t& cap, DevBuf<char>& dstage, hipStream_t st, bool parallel) {
    if (items.empty()) return hipSuccess;
    constexpr size_t kChunk = size_t{64} << 10;
    std::vector<CopyChunk> ch;
    for (const Item& it : items)
      for (size_t o = 0; o < it.bytes; o += kChunk)
        ch.push_back({reinterpret_cast<uint64_t>(static_cast<char*>(it.dev) + o), static_cast<uint32_t>((it.off + o) >> 8),
                      static_cast<uint32_t>(std::min(kChunk, it.bytes - o))});
    const size_t tb = (ch.size() * sizeof(CopyChunk) + 255) & ~size_t{255};
    const size_t all = tb + total;
    // chunk offsets are 256-byte units in 32 bits (items start 256-aligned,
    // chunks 64 KiB into them): staged plans up to 1 TiB
    if (total >= (size_t{1} << 40)) return hipErrorInvalidValue;
    if (all > cap) {
      if (buf) (void)hipHostFree(buf);
      buf = nullptr;
      cap = 0;
      const size_t want = all + all / 4;
      if (hipHostMalloc(reinterpret_cast<void**>(&buf), want, hipHostMallocPortable) != hipSuccess) {
        buf = nullptr;
        for (const auto& it : items) {   // pageable fallback
          const hipError_t e = hipMemcpyAsync(it.dev, it.host, it.bytes, hipMemcpyHostToDevice, st);
          if (e != hipSuccess) return e;
        }
        return hipSuccess;
      }
      cap = want;
    }
    hipError_t e = dstage.alloc(all);
    if (e != hipSuccess) return e;
    static const bool timing = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(buf, ch.data(), ch.size() * sizeof(CopyChunk));
    char* data = buf + tb;
    constexpr size_t kPiece = size_t{1} << 20;
    std::vector<std::pair<size_t, size_t>> pieces;   // (item, piece start)
    for (size_t i = 0; i < items.size(); ++i)
      for (size_t o = 0; o < items[i].bytes; o += kPiece) pieces.push_back({i, o});
    auto pack = [&](int64_t k0, int64_t k1) {
      for (int64_t k = k0; k < k1; ++k) {
        const Item& it = items[pieces[k].first];
        const size_t o = pieces[k].second, nb = std::min(kPiece, it.bytes - o);
        std::memcpy(data + it.off + o, static_cast<const char*>(it.host) + o, nb);
      }
    };
    if (parallel) parallel_chunks(static_cast<int64_t>(pieces.size()), 1, pack);
    else pack(0, static_cast<int64_t>(pieces.size()));
    const auto t1 = std::chrono::steady_clock::now();
    if ((e = hipMemcpyAsync(dstage.p, buf, all, hipMemcpyHostToDevice, st)) != hipSuccess) return e;
    launch_scatter_chunks(dstage.p + tb, reinterpret_cast<const CopyChunk*>(dstage.p), static_cast<int>(ch.size()), st);
    if (timing)
      std::fprintf(stderr, "[upload] %zu arrays, %zu chunks, %.2f MB: pack %.2f ms, enqueue %.2f ms\n", items.size(),
                   ch.size(), all / 1048576.0, std::chrono::duration<double, std::milli>(t1 - t0).count(),
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
    return hipGetLastError();
  }
};

struct GraphCopy {
  std::vector<uint64_t> keys[kNTypes];
  std::vector<double> meas[kNTypes], sig[kNTypes], hub[kNTypes];
  size_t n[kNTypes] = {};
  dynohip_graph_view view() const {
    dynohip_graph_view g;
    dynohip_factor_block* b[kNTypes] = {&g.pose_to_point, &g.landmark_motion_ternary, &g.between,
                                        &g.prior, &g.landmark_motion_pose, &g.landmark_pose_smoothing};
    for (int t = 0; t < kNTypes; ++t) {
      b[t]->n = n[t];
      b[t]->keys = keys[t].data();
      b[t]->measured = meas[t].empty() ? nullptr : meas[t].data();
      b[t]->sigmas = sig[t].data();
      b[t]->huber_k = hub[t].data();
    }
    return g;
  }
};

// The host side of a destroyed handle (its plan and graph copy) kept for the
// next handle: a full-batch call per frame creates a handle, plans, solves
// and destroys it, and freeing then re-faulting tens of MB of host arrays
// cost milliseconds each way (destroy 3.5 ms at C2). One slot; trimmed by
// dynohip_pool_trim.
struct HostCache {
  static HostCache& get() {
    static HostCache* c = new HostCache();
    return *c;
  }
  void give(Plan& p, GraphCopy& g) {
    std::lock_guard<std::mutex> lk(mu);
    if (has) return;
    plan = std::move(p);
    graph = std::move(g);
    has = true;
  }
  void take(Plan& p, GraphCopy& g) {
    std::lock_guard<std::mutex> lk(mu);
    if (!has) return;
    p = std::move(plan);
    g = std::move(graph);
    plan = Plan();
    graph = GraphCopy();
    has = false;
  }
  void trim() {
    std::lock_guard<std::mutex> lk(mu);
    plan = Plan();
    graph = GraphCopy();
    has = false;
  }
  std::mutex mu;
  Plan plan;
  GraphCopy graph;
  bool has = false;
};

struct TypeBufs {
  DevBuf<int32_t> idx;
  DevBuf<double> meas, isig, hk;
};

struct GatherBufs {
  DevBuf<int64_t> start;
  DevBuf<GEntry> ent;
  GatherDev dev(size_t nt) const {
    GatherDev g;
    g.n = static_cast<int>(nt);
    g.start = start.p;
    g.ent = ent.p;
    return g;
  }
};

}  // namespace

struct dynohip_solver {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t side = nullptr;       // update tasks of wide factorisation levels
  hipEvent_t ev_main = nullptr, ev_side = nullptr;
  std::string err;
  GraphCopy graph;
  bool has_graph = false;
  bool has_plan = false;
  // the plan's factor records (measurements, 1/sigma, Huber k) predate the
  // current graph, whose structure (factor keys per type) is the plan's
  bool records_stale = false;
  bool has_values = false;
  std::vector<uint64_t> value_keys;
  Plan plan;
  // device state
  DevBuf<double> pose, pt, pose_c, pt_c, arena;
  TypeBufs tb[kNTypes];
  TypeDev td[kNTypes];
  // fused static landmarks (k_lone_lin): k_linearize's view of the types
  // (PoseToPoint restricted to Plan::lin_list0) and the group kernel's
  TypeDev td_lin[kNTypes];
  DevBuf<int32_t> lin_list0;
  LoneLinDev lld;
  bool fused_env = true;   // DYNOHIP_FUSED_LONE=0 keeps the record path
  bool chain_lone = true;  // DYNOHIP_CHAIN_LONE=0: separate chain and lone-group launches
  GatherBufs gD, gE, gGp, gW, gRed, gGred;
  DevBuf<int32_t> redA, redB;
  DevBuf<uint32_t> redslot;
  DevBuf<int32_t> redorder;   // Plan::red_order (targets by entry count)
  DevBuf<int32_t> redblocks;  // Plan::red_blocks (the band blocks in column order)
  bool red_blocks_env = true; // DYNOHIP_RED_BLOCKS=0: each class's blocks in turn (A/B)
  DevBuf<int32_t> comp_start, comp_nb_start, nb_comp, nbedge_start, nbedge_pt, pt_edge_start, edge_pose, edge_pt;
  DevBuf<int64_t> comp_y_base;
  DevBuf<uint32_t> nbedge_w;
  DevBuf<int32_t> lone_blk;
  LoneSchurDev ld;
  DevBuf<double> slots, gred, xy, dpt, linv, contrib;
  DevBuf<int32_t> tile_pos, row_start, row_col, row_slot, bent, pairs;
  SmallMap smap{};  // the small solve's tile map (plans of <= kSmallNT tiles)
  DevBuf<TileTask> ftask;
  DevBuf<BackPart> bpart;
  bool small_solve = false; // DYNOHIP_SMALL_SOLVE=1: systems of <= kSmallNT tiles in one workgroup (at par with the DAG)
  DevBuf<double> bpartials;
  DevBuf<int> arrive;
  DevBuf<int32_t> fdep_start, fdep, fqueue;
  DevBuf<unsigned> fsync;   // [0] dataflow task queue head, [4..] per-slot write counters
  DevBuf<unsigned> done;
  DevBuf<double> partials, result;
  DevBuf<double> lcpart;     // block partials of the linearised cost change (k_backsub)
  DevBuf<unsigned> sumctr;   // arrival counter of the folded reductions
  // the linearised cost change: from the solve (k_backsub, default) or, with
  // DYNOHIP_LINERR_DIRECT=1 and on partitioned handles, as GTSAM forms it,
  // 0.5 ||J delta - b||^2 re-evaluated over the Jacobian records (k_linerr)
  bool linerr_direct = false;
  // inside `result`: doubles [0..3] results, [4] the solve's fail flag (int),
  // [5] the fail bits being accumulated (moved to [4] and cleared by the error sum)
  int* failp = nullptr;
  int partial_slots = 0;
  ChainDev cd;
  TileDev bd;
  TileSchedDev sd;
  // LM state
  dynohip_lm_params prm{};
  double lambda = 1e-5, error = 0.0;
  // `error` was computed by lm_reset at the current values and nothing has
  // moved them since (set_values then optimize: one initial error, not two)
  bool error_fresh = false;
  // the arena holds the linearisation at the current values (left there by
  // the speculative linearisation of an accepted step); next_oldlin is its
  // linear error at delta = 0
  bool lin_valid = false;
  // (the speculative linearisation's error at delta = 0, result[3], arrives
  // with the next try's results)
  // try results, copied into pinned host memory behind an event that is
  // recorded before the speculative linearisation is enqueued: the host
  // decides while the GPU linearises
  double* hres = nullptr;
  DevBuf<char> dstage[2];                 // device side of the upload staging
  char* stage[2] = {nullptr, nullptr};   // HandleRes::stage
  size_t stage_cap[2] = {0, 0};
  hipEvent_t ev_res = nullptr;
  int iterations = 0, inner = 0, converged = 0;
  std::vector<dynohip_trace_entry> trace;
  // values snapshot (bench hook), tagged with the plan it was taken under
  DevBuf<double> pose_snap, pt_snap;
  uint64_t plan_gen = 0, snap_gen = 0;   // snap_gen 0: no snapshot
  // phase timing (HIP events, optional)
  bool timing = false;
  hipEvent_t ev[9] = {};
  double phase_ms[7] = {};   // accumulated: lin, schur, assembly, chol, solve, backsub+linerr, retract+error
  int64_t n_lin = 0, n_solves = 0;
  dynohip_stats base_stats{};
  bool base_stats_valid = false;   // computed on first dynohip_get_stats after a re-plan
  // partitioned full-batch solve (partition.cpp): this handle is rank
  // `rank` of `nranks`; `comm` sums over ranks
  int nranks = 1, rank = 0;
  dynohip_allreduce_fn comm = nullptr;
  void* comm_ctx = nullptr;
  Partition part;
  GraphStore local_graph;
  std::vector<uint8_t> value_kind;   // global value kinds
  DevBuf<uint8_t> damp;
  // phase 0's right-hand-side move, and per separator phase (Plan::phases,
  // deepest node first) its tasks and right-hand-side move
  DevBuf<int32_t> seprhs_tile, seprhs_start, seprhs_slot;
  int n_seprhs = 0;
  struct PhaseDev {
    DevBuf<TileTask> ftask;
    DevBuf<int32_t> fdep_start, fdep, fqueue, rhs_tile, rhs_start, rhs_slot;
    TileSchedDev sd;
    int n_rhs = 0;
  };
  std::vector<std::unique_ptr<PhaseDev>> phd;
  DevBuf<double> xbuf;   // exchange buffer (the largest phase's)
  int64_t xtotal = 0;    // doubles exchanged per linear solve (every phase)
};

namespace {

int set_err(dynohip_solver* s, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  s->err = buf;
  return code;
}

#define HIPCHK(s, expr)                                                                     \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return set_err(s, DYNOHIP_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

int upload_gather(dynohip_solver* s, const GatherList& g, GatherBufs& b, Uploads& up) {
  HIPCHK(s, up.add(b.start, g.start));
  HIPCHK(s, up.add(b.ent, g.ent));
  return 0;
}

// types_done: the factor records were uploaded during planning (EarlyUpload)
int upload_plan(dynohip_solver* s, bool types_done = false) {
  Plan& P = s->plan;
  hipStream_t st = s->stream;
  Uploads up;
  HIPCHK(s, s->pose.alloc(12ull * P.n_pose));
  HIPCHK(s, s->pt.alloc(3ull * P.n_pt));
  HIPCHK(s, s->pose_c.alloc(12ull * P.n_pose));
  HIPCHK(s, s->pt_c.alloc(3ull * P.n_pt));
  HIPCHK(s, s->arena.alloc(P.arena_size));
  int slots = 1;
  for (int t = 0; t < kNTypes; ++t) {
    TypePlan& tp = P.types[t];
    if (!types_done) {
      HIPCHK(s, up.add(s->tb[t].idx, tp.idx));
      HIPCHK(s, up.add(s->tb[t].meas, tp.meas));
      HIPCHK(s, up.add(s->tb[t].isig, tp.isig));
      HIPCHK(s, up.add(s->tb[t].hk, tp.hk));
    }
    TypeDev& d = s->td[t];
    d.n = tp.n;
    d.base = tp.base;
    d.stride = tp.stride;
    d.idx = s->tb[t].idx.p;
    d.meas = s->tb[t].meas.p;
    d.isig = s->tb[t].isig.p;
    d.hk = s->tb[t].hk.p;
  }
  HIPCHK(s, up.add(s->lin_list0, P.lin_list0));
  for (int t = 0; t < kNTypes; ++t) s->td_lin[t] = s->td[t];
  s->td_lin[0].n = static_cast<int>(P.lin_list0.size());
  s->td_lin[0].list = s->lin_list0.p;
  LoneLinDev& ll = s->lld;
  ll.n_group = static_cast<int>(P.lgroup.size());
  ll.t0 = s->td[0];
  ll.off_W = P.off_W;
  ll.off_D = P.off_D;
  ll.off_gp = P.off_gp;
  slots = std::max(1, std::max(error_blocks(s->td), linearize_blocks(s->td_lin, &ll)));
  s->partial_slots = slots;
  HIPCHK(s, s->partials.alloc(2ull * slots));
  HIPCHK(s, s->result.alloc(8));
  HIPCHK(s, s->sumctr.alloc(1));
  HIPCHK(s, hipMemsetAsync(s->sumctr.p, 0, sizeof(unsigned), st));
  s->failp = reinterpret_cast<int*>(s->result.p + 5);
  HIPCHK(s, hipMemsetAsync(s->result.p, 0, 8 * sizeof(double), st));
  if (upload_gather(s, P.gD, s->gD, up) || upload_gather(s, P.gE, s->gE, up) || upload_gather(s, P.gGp, s->gGp, up) ||
      upload_gather(s, P.gW, s->gW, up) || upload_gather(s, P.gRed, s->gRed, up) ||
      upload_gather(s, P.gGred, s->gGred, up))
    return DYNOHIP_EHIP;
  HIPCHK(s, up.add(s->redA, P.red_A));
  HIPCHK(s, up.add(s->redB, P.red_B));
  HIPCHK(s, up.add(s->redslot, P.red_slot));
  {
    int64_t covered = 0;
    for (int c = 0; c < Plan::kRedClasses; ++c) covered += P.red_ncls[c];
    if (covered != static_cast<int64_t>(P.gRed.ntargets()) || P.red_order.size() != P.gRed.ntargets())
      return set_err(s, DYNOHIP_ESTRUCT, "internal: reduced-gather target classes do not cover the targets");
  }
  HIPCHK(s, up.add(s->redorder, P.red_order));
  HIPCHK(s, up.add(s->redblocks, P.red_blocks));
  HIPCHK(s, up.add(s->comp_start, P.comp_start));
  HIPCHK(s, up.add(s->comp_nb_start, P.comp_nb_start));
  HIPCHK(s, up.add(s->nb_comp, P.nb_comp));
  HIPCHK(s, up.add(s->comp_y_base, P.comp_y_base));
  HIPCHK(s, up.add(s->nbedge_start, P.nbedge_start));
  HIPCHK(s, up.add(s->nbedge_pt, P.nbedge_pt));
  HIPCHK(s, up.add(s->nbedge_w, P.nbedge_w));
  HIPCHK(s, up.add(s->pt_edge_start, P.pt_edge_start));
  HIPCHK(s, up.add(s->edge_pose, P.edge_pose));
  HIPCHK(s, up.add(s->edge_pt, P.edge_pt));
  HIPCHK(s, s->slots.alloc(static_cast<size_t>(P.n_slots) * kTile * kTile));
  HIPCHK(s, up.add(s->tile_pos, P.tile_pos));
  HIPCHK(s, up.add(s->row_start, P.row_start));
  HIPCHK(s, up.add(s->row_col, P.row_col));
  HIPCHK(s, up.add(s->row_slot, P.row_slot));
  HIPCHK(s, up.add(s->bent, P.bent));
  HIPCHK(s, up.add(s->ftask, P.ftask));
  HIPCHK(s, up.add(s->pairs, P.pairs));
  HIPCHK(s, s->contrib.alloc(static_cast<size_t>(P.n_slots) * kTile));
  HIPCHK(s, up.add(s->bpart, P.bpart));
  // (kept in the solver: Uploads packs the host arrays at up.run below)
  HIPCHK(s, s->bpartials.alloc(static_cast<size_t>(P.n_partials) * kTile + 1));
  HIPCHK(s, s->arrive.alloc(static_cast<size_t>(P.NT) + 1));
  HIPCHK(s, hipMemsetAsync(s->arrive.p, 0, (static_cast<size_t>(P.NT) + 1) * sizeof(int), st));
  HIPCHK(s, up.add(s->fdep_start, P.fdep_start));
  HIPCHK(s, up.add(s->fdep, P.fdep));
  HIPCHK(s, up.add(s->fqueue, P.fqueue));
  HIPCHK(s, s->fsync.alloc((static_cast<size_t>(P.n_slots) + 4 + 3) / 4 * 4));
  HIPCHK(s, hipMemsetAsync(s->fsync.p, 0, s->fsync.n * sizeof(unsigned), st));
  HIPCHK(s, s->done.alloc(static_cast<size_t>(P.NT) + 1));
  HIPCHK(s, hipMemsetAsync(s->done.p, 0, (static_cast<size_t>(P.NT) + 1) * sizeof(unsigned), st));
  s->sd.epoch = 0;
  const size_t nrp = static_cast<size_t>(P.NT) * kTile;
  HIPCHK(s, s->gred.alloc(nrp > 0 ? nrp : 1));
  HIPCHK(s, s->xy.alloc(2 * (nrp > 0 ? nrp : 1)));
  HIPCHK(s, s->linv.alloc(static_cast<size_t>(P.NT) * kTile * kTile + 1));
  HIPCHK(s, s->dpt.alloc(3ull * P.n_pt + 1));
  ChainDev& c = s->cd;
  c.n_comp = P.n_comp;
  c.n_nb = static_cast<int>(P.nb_pose.size());
  c.n_long = 0;
  while (c.n_long < P.n_comp && P.comp_start[c.n_long + 1] - P.comp_start[c.n_long] >= 2) ++c.n_long;
  c.n_nb_long = P.comp_nb_start.empty() ? 0 : P.comp_nb_start[c.n_long];
  c.comp_start = s->comp_start.p;
  c.comp_nb_start = s->comp_nb_start.p;
  c.nb_comp = s->nb_comp.p;
  c.comp_y_base = s->comp_y_base.p;
  c.nbedge_start = s->nbedge_start.p;
  c.nbedge_pt = s->nbedge_pt.p;
  c.nbedge_w = s->nbedge_w.p;
  c.pt_edge_start = s->pt_edge_start.p;
  c.edge_pose = s->edge_pose.p;
  c.edge_pt = s->edge_pt.p;
  // lone points (every chain after the long ones): their edges, and their Y
  // blocks, are contiguous in edge order (plan.cpp's lone-point layout)
  {
    const int32_t p0 = c.n_long < P.n_comp ? P.comp_start[c.n_long] : P.n_pt;
    c.e_lone0 = p0 < P.n_pt ? P.pt_edge_start[p0] : P.n_edge;
    // grouped lone points' Y is formed inside k_lone_schur and never stored
    c.n_lone_edges = P.lone_all_grouped ? 0 : P.n_edge - c.e_lone0;
    c.y_lone_base = c.n_long < P.n_comp ? static_cast<uint64_t>(P.comp_y_base[c.n_long]) : 0;
  }
  c.off_D = P.off_D;
  c.off_E = P.off_E;
  c.off_gp = P.off_gp;
  c.off_W = P.off_W;
  c.off_v = P.off_v;
  c.off_L = P.off_L;
  c.off_M = P.off_M;
  HIPCHK(s, up.add(s->lone_blk, P.lone_blk));
  LoneSchurDev& ld = s->ld;
  ld.n_group = static_cast<int>(P.lgroup.size());
  ld.blk = s->lone_blk.p;
  ld.max_m = P.lone_max_m;
  ld.off_W = P.off_W;
  ld.off_L = P.off_L;
  ld.off_gp = P.off_gp;
  ld.off_I6 = P.off_I6;
  ld.off_D = P.off_D;
  ld.off_v = P.off_v;
  s->lld.blk = s->lone_blk.p;
  HIPCHK(s, s->lcpart.alloc(static_cast<size_t>(backsub_blocks(
                                c, P.lone_all_grouped ? static_cast<int>(P.lgroup.size()) : 0, P.n_pose)) + 1));
  TileDev& b = s->bd;
  b.NT = P.NT;
  b.n_red = P.n_red;
  b.slots = s->slots.p;
  b.pos = s->tile_pos.p;
  b.row_start = s->row_start.p;
  b.row_col = s->row_col.p;
  b.row_slot = s->row_slot.p;
  if (P.NT >= 1 && P.NT <= kSmallNT) {
    SmallMap& m = s->smap;
    for (int t = 0; t < P.NT; ++t) m.ord[P.tile_pos[t]] = t;
    for (int p = 0; p < P.NT; ++p)
      for (int q = 0; q < P.NT; ++q) {
        int32_t sl = -1;
        if (p <= q)
          for (int e = P.row_start[m.ord[q]]; e < P.row_start[m.ord[q] + 1]; ++e)
            if (P.row_col[e] == m.ord[p]) sl = P.row_slot[e];
        m.slot[p][q] = sl;
      }
  }
  s->sd.ftask = s->ftask.p;
  s->sd.pairs = s->pairs.p;
  s->sd.bpart = s->bpart.p;
  s->sd.partials = s->bpartials.p;
  s->sd.arrive = s->arrive.p;
  s->sd.done = s->done.p;
  s->sd.bent = s->bent.p;
  s->sd.fdep_start = s->fdep_start.p;
  s->sd.fdep = s->fdep.p;
  s->sd.forder = s->fqueue.p;
  s->sd.fqueue = s->fsync.p;
  s->sd.wcnt = s->fsync.p + 4;
  HIPCHK(s, up.run(s->stage[1], s->stage_cap[1], s->dstage[1], st, true));
  // debug: DYNOHIP_POISON_MASK fills the selected device buffers with NaN
  // bytes after a re-plan (bit 0 arena, 1 partials, 2 slots, 3 gred, 4 xy,
  // 5 dpt, (6 unused), 7 linv, 8 contrib, 9 bpartials, 10 pose_c/pt_c), so a read
  // of a never-written element shows up
  if (const char* pm = std::getenv("DYNOHIP_POISON_MASK")) {
    const unsigned mask = static_cast<unsigned>(std::strtoul(pm, nullptr, 0));
    auto poison = [&](unsigned bit, void* p, size_t bytes) {
      if ((mask >> bit) & 1u && p && bytes) (void)hipMemsetAsync(p, 0xff, bytes, st);
    };
    poison(0, s->arena.p, s->arena.n * 8);
    poison(1, s->partials.p, s->partials.n * 8);
    poison(2, s->slots.p, s->slots.n * 8);
    poison(3, s->gred.p, s->gred.n * 8);
    poison(4, s->xy.p, s->xy.n * 8);
    poison(5, s->dpt.p, s->dpt.n * 8);
    poison(7, s->linv.p, s->linv.n * 8);
    poison(8, s->contrib.p, s->contrib.n * 8);
    poison(9, s->bpartials.p, s->bpartials.n * 8);
    poison(10, s->pose_c.p, s->pose_c.n * 8);
    poison(10, s->pt_c.p, s->pt_c.n * 8);
  }
  HIPCHK(s, hipStreamSynchronize(st));
  return 0;
}

int upload_partition(dynohip_solver* s) {
  Plan& P = s->plan;
  hipStream_t st = s->stream;
  HIPCHK(s, s->damp.upload(s->part.damp_row, st));
  s->n_seprhs = static_cast<int>(P.rhs0_tile.size());
  HIPCHK(s, s->seprhs_tile.upload(P.rhs0_tile, st));
  HIPCHK(s, s->seprhs_start.upload(P.rhs0_start, st));
  HIPCHK(s, s->seprhs_slot.upload(P.rhs0_slot, st));
  while (s->phd.size() < P.phases.size()) s->phd.push_back(std::make_unique<dynohip_solver::PhaseDev>());
  s->xtotal = 0;
  size_t nx = 0;
  for (size_t ph = 0; ph < P.phases.size(); ++ph) {
    const PartPhase& F = P.phases[ph];
    dynohip_solver::PhaseDev& D = *s->phd[ph];
    HIPCHK(s, D.ftask.upload(F.ftask, st));
    HIPCHK(s, D.fdep_start.upload(F.fdep_start, st));
    HIPCHK(s, D.fdep.upload(F.fdep, st));
    HIPCHK(s, D.fqueue.upload(F.fqueue, st));
    HIPCHK(s, D.rhs_tile.upload(F.rhs_tile, st));
    HIPCHK(s, D.rhs_start.upload(F.rhs_start, st));
    HIPCHK(s, D.rhs_slot.upload(F.rhs_slot, st));
    D.n_rhs = static_cast<int>(F.rhs_tile.size());
    D.sd = s->sd;
    D.sd.ftask = D.ftask.p;
    D.sd.fdep_start = D.fdep_start.p;
    D.sd.fdep = D.fdep.p;
    D.sd.forder = D.fqueue.p;
    size_t n = 0;
    for (size_t r = 0; r + 1 < F.xslot.size(); r += 2)
      n += static_cast<size_t>(F.xslot[r + 1] - F.xslot[r]) * kTile * kTile;
    for (size_t r = 0; r + 1 < F.xtile.size(); r += 2) n += static_cast<size_t>(F.xtile[r + 1] - F.xtile[r]) * kTile;
    nx = std::max(nx, n);
    s->xtotal += static_cast<int64_t>(n);
  }
  HIPCHK(s, s->xbuf.alloc(nx));
  // rows and contributions of other ranks' interiors and separators are
  // never written here: keep them zero (their poses then retract by zero)
  HIPCHK(s, hipMemsetAsync(s->contrib.p, 0, s->contrib.n * sizeof(double), st));
  HIPCHK(s, hipMemsetAsync(s->xy.p, 0, s->xy.n * sizeof(double), st));
  HIPCHK(s, hipStreamSynchronize(st));
  return 0;
}

// sum over ranks (partitioned); no-op on an ordinary handle
int comm_sum(dynohip_solver* s, double* buf, size_t n, int on_device) {
  if (s->nranks <= 1 || n == 0) return 0;
  if (!s->comm || s->comm(s->comm_ctx, buf, n, on_device, static_cast<void*>(s->stream)) != 0)
    return set_err(s, DYNOHIP_EHIP, "partition exchange (all-reduce of %zu doubles) failed", n);
  return 0;
}

// copies one depth's separator tiles and RHS rows (phase ph's exchange)
// into / out of the exchange buffer
int sep_copy(dynohip_solver* s, size_t ph, bool pack, size_t* n_out = nullptr) {
  const PartPhase& F = s->plan.phases[ph];
  size_t o = 0;
  auto cp = [&](double* dev, size_t cnt) -> int {
    double* a = pack ? s->xbuf.p + o : dev;
    const double* b = pack ? dev : s->xbuf.p + o;
    HIPCHK(s, hipMemcpyAsync(a, b, cnt * sizeof(double), hipMemcpyDeviceToDevice, s->stream));
    o += cnt;
    return 0;
  };
  for (size_t r = 0; r + 1 < F.xslot.size(); r += 2)
    if (cp(s->slots.p + static_cast<size_t>(F.xslot[r]) * kTile * kTile,
           static_cast<size_t>(F.xslot[r + 1] - F.xslot[r]) * kTile * kTile))
      return DYNOHIP_EHIP;
  for (size_t r = 0; r + 1 < F.xtile.size(); r += 2)
    if (cp(s->gred.p + static_cast<size_t>(F.xtile[r]) * kTile,
           static_cast<size_t>(F.xtile[r + 1] - F.xtile[r]) * kTile))
      return DYNOHIP_EHIP;
  if (n_out) *n_out = o;
  return 0;
}

// error at (pose, pt) into result[slot]
// extra_n > 0: the finishing block also sums the cost-change partials of the
// back-substitution into result[0] (lin_change_mode)
void enqueue_error(dynohip_solver* s, const double* pose, const double* pt, double* partials, double* out,
                   int extra_n = 0) {
  launch_error(s->td, pose, pt, partials, s->sumctr.p, out, s->failp, reinterpret_cast<int*>(s->result.p + 4),
               s->stream, s->lcpart.p, extra_n, extra_n > 0 ? s->result.p : nullptr);
}

void enqueue_linerr(dynohip_solver* s, const double* dpose, const double* dpt, double* partials, double* out) {
  launch_linerr(s->td, s->arena.p, dpose, dpt, partials, s->sumctr.p, out, s->stream);
}

int compute_error(dynohip_solver* s, const double* pose, const double* pt, double* err_out) {
  enqueue_error(s, pose, pt, s->partials.p, s->result.p);
  HIPCHK(s, hipMemcpyAsync(err_out, s->result.p, sizeof(double), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  return comm_sum(s, err_out, 1, 0);
}

// result[0] of a try holds the linearised cost change (x2) rather than the
// new linear error
bool lin_change_mode(const dynohip_solver* s) { return s->nranks == 1 && !s->linerr_direct; }

// The static landmarks are linearised inside their group blocks (k_lone_lin),
// with no Jacobian record: every lone point grouped, and nothing reading the
// records afterwards (the direct linear error and the partitioned handles do)
bool fused_lone(const dynohip_solver* s) {
  return s->fused_env && s->plan.lone_all_grouped && !s->plan.lgroup.empty() && lin_change_mode(s);
}

// linearisation + point-side blocks (once per outer iteration); lin0, when
// given, receives the linear error at delta = 0 (0.5 ||b||^2).
// all_records: every factor's J | b record (the dynohip_linearize test hook)
int enqueue_linearize(dynohip_solver* s, const double* pose, const double* pt, double* lin0 = nullptr,
                      bool all_records = false) {
  Plan& P = s->plan;
  double* A = s->arena.p;
  const GatherDev g[4] = {s->gD.dev(P.gD.ntargets()), s->gE.dev(P.gE.ntargets()), s->gGp.dev(P.gGp.ntargets()),
                          s->gW.dev(P.gW.ntargets())};
  double* const dst[4] = {A + P.off_D, A + P.off_E, A + P.off_gp, A + P.off_W};
  if (fused_lone(s) && !all_records) {
    if (launch_linearize(s->td_lin, pose, pt, A, s->partials.p, s->sumctr.p, lin0, s->stream, &s->lld))
      return set_err(s, DYNOHIP_EHIP, "internal: fused static-landmark linearisation without its tables");
    launch_gather_point(g, dst, A, s->stream);
    return 0;
  }
  launch_linearize(s->td, pose, pt, A, s->partials.p, s->sumctr.p, lin0, s->stream);
  launch_gather_point(g, dst, A, s->stream, P.lone_all_grouped ? static_cast<int>(P.lgroup.size()) : 0,
                      s->lone_blk.p);
  return 0;
}

// damped solve + linearised error + retract + error for one lambda.
// result[0] = new linear error (or 2x the cost change, lin_change_mode),
// result[1] = new nonlinear error; fail flag.
int enqueue_try(dynohip_solver* s, double lambda) {
  const bool timed = s->timing;
  Plan& P = s->plan;
  hipStream_t st = s->stream;
  double* A = s->arena.p;
  const size_t nrp = static_cast<size_t>(P.NT) * kTile;
  if (timed) (void)hipEventRecord(s->ev[2], st);
  ZeroDev z;
  z.p[0] = s->slots.p;
  z.n[0] = static_cast<int64_t>(P.n_slots) * kTile * kTile;
  z.p[1] = s->gred.p;
  z.n[1] = static_cast<int64_t>(nrp);
  z.p[2] = reinterpret_cast<double*>(s->fsync.p);
  z.n[2] = static_cast<int64_t>(s->fsync.n) / 2;
  if (s->sd.back_poll) {   // k_back_poll's hand-off buffers
    z.s[0] = s->xy.p + nrp;
    z.sn[0] = static_cast<int64_t>(nrp);
    z.s[1] = s->bpartials.p;
    z.sn[1] = static_cast<int64_t>(P.n_partials) * kTile;
  }
  s->ld.fused = fused_lone(s) ? 1 : 0;
  if (P.lone_all_grouped && !P.lgroup.empty() && s->chain_lone) {
    // the groups factor their own points beside the chain recurrences
    launch_chain_lone(s->cd, s->ld, A, lambda, s->failp, z, st);
    launch_chain_solve_y(s->cd, A, st);
  } else {
    launch_chain_factor(s->cd, A, lambda, s->failp, z, st);
    launch_chain_solve_y(s->cd, A, st);
    launch_lone_schur(s->ld, A, st);
  }
  if (timed) (void)hipEventRecord(s->ev[3], st);
  launch_gather_reduced(s->gRed.dev(P.gRed.ntargets()), s->redorder.p, P.red_ncls, s->redA.p, s->redB.p, s->redslot.p,
                        s->gGred.dev(P.gGred.ntargets()),
                        s->gred.p, A, s->bd, lambda, st, s->nranks > 1 ? s->damp.p : nullptr,
                        s->red_blocks_env && !P.red_blocks.empty() ? s->redblocks.p : nullptr,
                        static_cast<int>(P.red_blocks.size()));
  if (timed) (void)hipEventRecord(s->ev[4], st);
  double* y = s->xy.p;
  double* x = s->xy.p + nrp;
  if (++s->sd.epoch == 0) s->sd.epoch = 1;  // stamps of earlier solves never match
  if (s->nranks > 1) {
    // phase 0: this rank's subtree and its updates of the separator tiles;
    // its interior contributions leave the separator RHS rows
    launch_tile_forward(s->bd, s->sd, P.flevel, P.fpanels, s->linv.p, s->gred.p, s->contrib.p, y, s->failp, st,
                        s->side, s->ev_main, s->ev_side);
    launch_sep_rhs(s->n_seprhs, s->seprhs_tile.p, s->seprhs_start.p, s->seprhs_slot.p, s->gred.p, s->contrib.p, 1, st);
    // then this rank's separator nodes, deepest first: the exchange of the
    // node's depth (its separator systems summed over ranks, ordered on the
    // solver's stream by the callback: no host synchronisation here), the
    // node's tasks on its group, its contributions to the separators above
    // into their RHS rows (leader) or dropped (the group's other ranks)
    for (size_t ph = 0; ph < P.phases.size(); ++ph) {
      size_t nxd = 0;
      if (sep_copy(s, ph, true, &nxd)) return DYNOHIP_EHIP;
      int rc = comm_sum(s, s->xbuf.p, nxd, 1);
      if (rc) return rc;
      if (sep_copy(s, ph, false)) return DYNOHIP_EHIP;
      HIPCHK(s, hipMemsetAsync(s->fsync.p, 0, s->fsync.n * sizeof(unsigned), st));
      dynohip_solver::PhaseDev& D = *s->phd[ph];
      D.sd.epoch = s->sd.epoch;
      launch_tile_forward(s->bd, D.sd, P.phases[ph].flevel, P.phases[ph].fpanels, s->linv.p, s->gred.p, s->contrib.p,
                          y, s->failp, st, s->side, s->ev_main, s->ev_side);
      launch_sep_rhs(D.n_rhs, D.rhs_tile.p, D.rhs_start.p, D.rhs_slot.p, s->gred.p, s->contrib.p, P.phases[ph].leader,
                     st);
    }
    // (ms_cholesky of a partitioned handle spans every forward phase and the
    // exchanges between them)
    if (timed) (void)hipEventRecord(s->ev[5], st);
    launch_tile_backward(s->bd, s->sd, P.bplevel, s->linv.p, y, x, s->failp, st, s->sd.back_poll);
  } else if (s->small_solve && P.NT >= 1 && P.NT <= kSmallNT) {
    // a window-sized system: factorisation and both substitutions in one
    // workgroup (k_small_solve; ms_cholesky spans all of it)
    launch_small_solve(s->bd, s->smap, s->gred.p, x, s->failp, st);
    if (timed) (void)hipEventRecord(s->ev[5], st);
  } else {
    launch_tile_forward(s->bd, s->sd, P.flevel, P.fpanels, s->linv.p, s->gred.p, s->contrib.p, y, s->failp, st,
                        s->side, s->ev_main, s->ev_side);
    if (timed) (void)hipEventRecord(s->ev[5], st);
    launch_tile_backward(s->bd, s->sd, P.bplevel, s->linv.p, y, x, s->failp, st, s->sd.back_poll);
  }
  if (timed) (void)hipEventRecord(s->ev[6], st);
  // pose deltas are x[0 .. 6 n_pose) in pose-index order
  const int n_lone = P.lone_all_grouped ? static_cast<int>(P.lgroup.size()) : 0;
  if (lin_change_mode(s)) {
    // result[0] = delta^T g + lambda ||delta||^2 (twice the linearised cost change)
    // (and the candidate values: pose_c, pt_c)
    LinChangeDev lc;
    lc.partials = s->lcpart.p;
    lc.out = s->result.p;
    lc.gred = s->gred.p;
    lc.n_pose = P.n_pose;
    lc.lambda = lambda;
    lc.pose = s->pose.p;
    lc.pt = s->pt.p;
    lc.pose_out = s->pose_c.p;
    lc.pt_out = s->pt_c.p;
    launch_backsub(s->cd, A, x, s->dpt.p, st, n_lone, s->lone_blk.p, &lc);
  } else {
    // result[0] = the linear error at delta
    launch_backsub(s->cd, A, x, s->dpt.p, st, n_lone, s->lone_blk.p);
    enqueue_linerr(s, x, s->dpt.p, s->partials.p, s->result.p);
  }
  if (timed) (void)hipEventRecord(s->ev[7], st);
  const int nlc = lin_change_mode(s) ? backsub_blocks(s->cd, n_lone, P.n_pose) : 0;
  if (!lin_change_mode(s)) launch_retract(P.n_pose, P.n_pt, s->pose.p, s->pt.p, x, s->dpt.p, s->pose_c.p, s->pt_c.p, st);
  else if (nlc == 0) HIPCHK(s, hipMemsetAsync(s->result.p, 0, sizeof(double), st));
  enqueue_error(s, s->pose_c.p, s->pt_c.p, s->partials.p + s->partial_slots, s->result.p + 1, nlc);
  if (timed) (void)hipEventRecord(s->ev[8], st);
  return 0;
}

void push_trace(dynohip_solver* s, const dynohip_trace_entry& e) { s->trace.push_back(e); }

// algorithmic work per linearisation / assembly / factorisation
void compute_base_stats(dynohip_solver* s) {
  const Plan& P = s->plan;
  dynohip_stats& st = s->base_stats;
  std::memset(&st, 0, sizeof(st));
  st.n_pose = P.n_pose;
  st.n_point = P.n_pt;
  st.n_chain = P.n_comp;
  st.n_edge = P.n_edge;
  st.reduced_dim = P.n_red;
  st.tiles_stored = P.n_slots;
  st.band_max_tiles = P.max_D;
  st.chol_levels = P.flevel.empty() ? 0 : static_cast<int64_t>(P.flevel.size()) - 1;
  st.back_levels = P.blevel.empty() ? 0 : static_cast<int64_t>(P.blevel.size()) - 1;
  st.nd_leaf = P.nd_leaf;
  // SURVEY.md §8(d) B_A: what one Jacobian assembly must read and write
  double rd = 96.0 * P.n_pose + 24.0 * P.n_pt, impl = 0.0;
  std::vector<uint64_t> pp;   // distinct pose-pose pairs of multi-pose factors
  for (int t = 0; t < kNTypes; ++t) {
    const TypePlan& tp = P.types[t];
    st.n_factor += tp.n;
    rd += (4.0 * kNKeys[t] + 8.0 * kMeasDim[t]) * tp.n;
    // the record implementation: indices, measurement, 1/sigma and Huber k
    // and the slot values read, the J | b record written, then re-read by
    // the point-side gathers
    double per = 4.0 * kNKeys[t] + 8.0 * kMeasDim[t] + 8.0 * kDim[t] + 8.0 + 2.0 * 8.0 * tp.stride;
    for (int sl = 0; sl < kNKeys[t]; ++sl) per += kSlotKind[t][sl] == 0 ? 96.0 : 24.0;
    if (t == 0 && fused_lone(s)) {
      // the grouped static landmarks' factors (k_lone_lin) read their inputs
      // and write no record
      const double nrec = static_cast<double>(P.lin_list0.size());
      impl += per * nrec + (per - 2.0 * 8.0 * tp.stride) * (tp.n - nrec);
    } else {
      impl += per * tp.n;
    }
    for (int i = 0; i < tp.n; ++i)
      for (int a = 0; a < kNKeys[t]; ++a)
        for (int b = a + 1; b < kNKeys[t]; ++b)
          if (kSlotKind[t][a] == 0 && kSlotKind[t][b] == 0) {
            const uint64_t x = static_cast<uint32_t>(tp.idx[static_cast<size_t>(i) * kNKeys[t] + a]);
            const uint64_t y = static_cast<uint32_t>(tp.idx[static_cast<size_t>(i) * kNKeys[t] + b]);
            pp.push_back(x < y ? (x << 32 | y) : (y << 32 | x));
          }
  }
  std::sort(pp.begin(), pp.end());
  const double n_pp = static_cast<double>(std::unique(pp.begin(), pp.end()) - pp.begin());
  const double wr = 8.0 * (9.0 * P.n_pt + 18.0 * P.n_edge + 9.0 * P.gE.ntargets() + 27.0 * P.n_pose + 36.0 * n_pp);
  st.lin_bytes = rd + wr;
  st.lin_bytes_read = rd;
  // point-side block outputs (D, E, g_p, W) written by the gathers; the
  // fused groups' H areas (42 doubles per group and neighbour)
  impl += 8.0 * (9.0 * P.n_pt + 9.0 * P.gE.ntargets() + 3.0 * P.n_pt + 18.0 * P.n_edge);
  if (fused_lone(s))
    for (const LoneGroup& G : P.lgroup) impl += 8.0 * 42.0 * G.m;
  st.lin_bytes_impl = impl;
  // the reduced assembly: every entry descriptor (16 B), every distinct
  // operand block once (a block feeding several targets is counted once: the
  // re-reads are L2 hits, not algorithmic bytes) and every output written
  double asmb = 0.0;
  {
    std::vector<uint64_t> blk;   // (arena offset << 8) | doubles
    blk.reserve(2 * (P.gRed.ent.size() + P.gGred.ent.size()));
    auto add = [&](uint32_t off, int nd) { blk.push_back((static_cast<uint64_t>(off) << 8) | static_cast<uint64_t>(nd)); };
    for (const GEntry& e : P.gRed.ent) {
      if (e.sign == kAddBlock) {
        add(e.b, 36);
      } else {
        add(e.a, 6 * e.k);
        add(e.b, 6 * e.k);
      }
    }
    for (const GEntry& e : P.gGred.ent) {
      if (e.sign == kAddBlock) {
        add(e.b, 6);
      } else {
        add(e.a, 6 * e.k);
        add(e.b, e.k);
      }
    }
    std::sort(blk.begin(), blk.end());
    blk.erase(std::unique(blk.begin(), blk.end()), blk.end());
    for (uint64_t x : blk) asmb += 8.0 * static_cast<double>(x & 0xffu);
    asmb += 16.0 * static_cast<double>(P.gRed.ent.size() + P.gGred.ent.size());
  }
  asmb += 36.0 * 8.0 * P.gRed.ntargets() + 6.0 * 8.0 * P.n_pose;
  st.assembly_bytes = asmb;
  // envelope Cholesky flop count of the reduced system
  std::vector<int32_t> firstpose(P.n_pose);
  for (int a = 0; a < P.n_pose; ++a) firstpose[a] = a;
  for (size_t t = 0; t < P.red_A.size(); ++t)
    firstpose[P.red_A[t]] = std::min(firstpose[P.red_A[t]], P.red_B[t]);
  // rows of a pose share f_i; flops(i, j) = 2 * (j - max(f_i, f_j)) (+ 1)
  double fl = 0.0;
  for (int a = 0; a < P.n_pose; ++a) {
    const int64_t fi = 6ll * firstpose[a];
    for (int r = 0; r < 6; ++r) {
      const int64_t i = 6ll * a + r;
      for (int64_t j = fi; j <= i; ++j) {
        const int64_t fj = 6ll * firstpose[j / 6];
        fl += 2.0 * static_cast<double>(j - std::max(fi, fj)) + 1.0;
      }
    }
  }
  st.chol_flops = fl;
  st.chol_tile_flops = P.tile_flops;
}

// LevenbergMarquardtOptimizer::iterate()
int lm_iterate(dynohip_solver* s) {
  hipStream_t st = s->stream;
  s->error_fresh = false;
  // Speculation: right after each try, the linearisation at the candidate
  // values is enqueued too (before the host has seen whether the step is
  // accepted), so the GPU is not idle while the host decides. Accepted: the
  // arena already holds the next iteration's linearisation. Rejected: the
  // current values are re-linearised before the next try. Results are
  // identical either way; phase timing runs without speculation.
  const bool speculate = !s->timing;
  double oldLin = 0.0;
  bool have_old = false;
  int oldlin_slot = 2;   // result[] slot of the linear error at delta = 0
  if (s->lin_valid) {
    oldlin_slot = 3;
  } else {
    if (s->timing) (void)hipEventRecord(s->ev[0], st);
    if (int rc = enqueue_linearize(s, s->pose.p, s->pt.p, s->result.p + 2)) return rc;
    if (s->timing) (void)hipEventRecord(s->ev[1], st);
  }
  s->lin_valid = false;
  s->n_lin++;
  bool relinearize = false;
  for (;;) {
    dynohip_trace_entry te{};
    te.outer_iteration = s->iterations;
    te.lambda = s->lambda;
    te.current_error = s->error;
    te.new_error = INFINITY;
    te.old_linear_error = oldLin;
    if (relinearize) {
      // a rejected speculative step left the candidate's linearisation
      if (int rc = enqueue_linearize(s, s->pose.p, s->pt.p)) return rc;
      s->n_lin++;
      relinearize = false;
    }
    int trc = enqueue_try(s, s->lambda);
    if (trc) return trc;
    HIPCHK(s, hipMemcpyAsync(s->hres, s->result.p, 5 * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(s, hipEventRecord(s->ev_res, st));
    if (speculate) {
      // result[3] is read with the next try's results (stream order keeps
      // this launch's value until then)
      if (int rc = enqueue_linearize(s, s->pose_c.p, s->pt_c.p, s->result.p + 3)) return rc;
    }
    HIPCHK(s, hipEventSynchronize(s->ev_res));
    double res[5];
    std::memcpy(res, s->hres, sizeof(res));
    int fail = 0;
    std::memcpy(&fail, &res[4], sizeof(int));
    if (s->nranks > 1) {
      // errors are sums over the ranks' factors; fail bits are OR-ed
      double red[8] = {res[0], res[1], res[2], res[3], (fail & 1) ? 1.0 : 0.0, (fail & 2) ? 1.0 : 0.0,
                       (fail & 4) ? 1.0 : 0.0, 0.0};
      int rc = comm_sum(s, red, 8, 0);
      if (rc) return rc;
      for (int k = 0; k < 4; ++k) res[k] = red[k];
      fail = (red[4] > 0 ? 1 : 0) | (red[5] > 0 ? 2 : 0) | (red[6] > 0 ? 4 : 0);
    }
    if (!have_old) {
      oldLin = res[oldlin_slot];
      te.old_linear_error = oldLin;
      have_old = true;
      if (s->timing) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, s->ev[0], s->ev[1]);
        s->phase_ms[0] += ms;
      }
    }
    s->n_solves++;
    if (s->timing) {
      float ms = 0.f;
      for (int k = 2; k < 8; ++k) {
        (void)hipEventElapsedTime(&ms, s->ev[k], s->ev[k + 1]);
        s->phase_ms[k - 1] += ms;
      }
    }
    if (fail & 2) return set_err(s, DYNOHIP_EHIP, "backward solve: dependency wait timed out");
    if (fail & 4) return set_err(s, DYNOHIP_EHIP, "factorisation: dependency wait timed out");
    const int solved = fail == 0 && std::isfinite(res[0]);
    te.solved = solved;
    bool step_ok = false, stop = false;
    double modelFidelity = 0.0, newError = INFINITY;
    if (solved) {
      // linearizedCostChange (LevenbergMarquardtOptimizer.cpp tryLambda): from
      // the solve, or oldLinearizedError - newLinearizedError as GTSAM forms it
      const bool from_solve = lin_change_mode(s);
      const double linChange = from_solve ? 0.5 * res[0] : oldLin - res[0];
      const double newLin = from_solve ? oldLin - linChange : res[0];
      te.new_linear_error = newLin;
      if (linChange >= 0) {
        newError = res[1];
        te.new_error = newError;
        const double costChange = s->error - newError;
        if (linChange > DBL_EPSILON * oldLin) {
          modelFidelity = costChange / linChange;
          step_ok = modelFidelity > s->prm.min_model_fidelity;
        }
        if (std::fabs(costChange) < s->prm.relative_error_tol * s->error) stop = true;
      }
    }
    te.model_fidelity = modelFidelity;
    te.accepted = step_ok;
    te.stop = stop;
    push_trace(s, te);
    if (step_ok) {
      s->pose.swap(s->pose_c);
      s->pt.swap(s->pt_c);
      if (speculate) s->lin_valid = true;
      s->error = newError;
      s->lambda /= s->prm.lambda_factor;
      if (s->lambda < s->prm.lambda_lower_bound) s->lambda = s->prm.lambda_lower_bound;
      s->iterations++;
      s->inner++;
      break;
    } else if (!stop) {
      s->lambda *= s->prm.lambda_factor;
      s->inner++;
      if (s->lambda >= s->prm.lambda_upper_bound) break;
      relinearize = speculate;
    } else {
      break;
    }
  }
  return 0;
}

void fill_summary(const dynohip_solver* s, double initial, dynohip_lm_summary* out) {
  if (!out) return;
  out->iterations = s->iterations;
  out->inner_iterations = s->inner;
  out->initial_error = initial;
  out->final_error = s->error;
  out->final_lambda = s->lambda;
  out->converged = s->converged;
  out->reserved = 0;
}

int ready(dynohip_solver* s) {
  if (!s) return DYNOHIP_EINVAL;
  if (!s->has_graph || !s->has_plan || !s->has_values) return set_err(s, DYNOHIP_ESTATE, "graph and values must be set");
  return 0;
}

}  // namespace

// ======================================================================
extern "C" {

int dynohip_abi_version(void) { return DYNOHIP_ABI_VERSION; }

void dynohip_lm_params_default(dynohip_lm_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->lambda_initial = 1e-5;
  p->lambda_factor = 10.0;
  p->lambda_upper_bound = 1e5;
  p->lambda_lower_bound = 0.0;
  p->min_model_fidelity = 1e-3;
  p->relative_error_tol = 1e-5;
  p->absolute_error_tol = 1e-5;
  p->error_tol = 0.0;
  p->max_iterations = 100;
  p->diagonal_damping = 0;
  p->use_fixed_lambda_factor = 1;
}

int dynohip_create(int device_id, dynohip_solver** out) {
  if (!out) return DYNOHIP_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return DYNOHIP_EHIP;
  if (device_id < 0 || device_id >= ndev) return DYNOHIP_EINVAL;
  if (hipSetDevice(device_id) != hipSuccess) return DYNOHIP_EHIP;
  HandleRes r;
  if (!ResPool::get().take(device_id, &r)) {
    r.device = device_id;
    // (the second stream of the level-launched factorisation is made when
    // that path is chosen, dynohip_set_exec_options: a stream takes one of
    // the process's few hardware queues, which several handles driven from
    // several threads -- deferred sliding windows -- need for their own)
    bool ok = hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&r.ev_main, hipEventDisableTiming) == hipSuccess &&
              hipEventCreateWithFlags(&r.ev_res, hipEventDisableTiming) == hipSuccess &&
              hipHostMalloc(reinterpret_cast<void**>(&r.hres), 8 * sizeof(double), hipHostMallocDefault) == hipSuccess;
    for (auto& e : r.ev) ok = ok && hipEventCreate(&e) == hipSuccess;
    if (!ok) {
      for (auto& e : r.ev)
        if (e) (void)hipEventDestroy(e);
      if (r.ev_res) (void)hipEventDestroy(r.ev_res);
      if (r.ev_main) (void)hipEventDestroy(r.ev_main);
      if (r.ev_side) (void)hipEventDestroy(r.ev_side);
      if (r.hres) (void)hipHostFree(r.hres);
      if (r.side) (void)hipStreamDestroy(r.side);
      if (r.stream) (void)hipStreamDestroy(r.stream);
      return DYNOHIP_EHIP;
    }
  }
  dynohip_solver* s = new dynohip_solver();
  HostCache::get().take(s->plan, s->graph);   // stale contents: has_graph / has_plan are false
  s->device = device_id;
  if (const char* e = std::getenv("DYNOHIP_LINERR_DIRECT")) s->linerr_direct = std::atoi(e) != 0;
  if (const char* e = std::getenv("DYNOHIP_FUSED_LONE")) s->fused_env = std::atoi(e) != 0;
  if (const char* e = std::getenv("DYNOHIP_BACK_POLL")) s->sd.back_poll = std::atoi(e) != 0;
  if (const char* e = std::getenv("DYNOHIP_CHAIN_LONE")) s->chain_lone = std::atoi(e) != 0;
  if (const char* e = std::getenv("DYNOHIP_SMALL_SOLVE")) s->small_solve = std::atoi(e) != 0;
  if (const char* e = std::getenv("DYNOHIP_RED_BLOCKS")) s->red_blocks_env = std::atoi(e) != 0;
  s->stream = r.stream;
  s->side = r.side;
  s->ev_main = r.ev_main;
  s->ev_side = r.ev_side;
  s->ev_res = r.ev_res;
  for (int k = 0; k < 9; ++k) s->ev[k] = r.ev[k];
  s->hres = r.hres;
  for (int k = 0; k < 2; ++k) {
    s->stage[k] = r.stage[k];
    s->stage_cap[k] = r.stage_cap[k];
  }
  // the dataflow factorisation keeps one 158 KB-LDS workgroup per CU
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device_id) == hipSuccess && cus > 0)
    s->sd.workers = cus;
  dynohip_lm_params_default(&s->prm);
  *out = s;
  return DYNOHIP_OK;
}

// The handle's streams, events and pinned buffer go back to ResPool and its
// device buffers to DevPool (see DevPool): destroying a handle frees nothing
// and synchronises only its own streams.
void dynohip_destroy(dynohip_solver* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  if (s->side) (void)hipStreamSynchronize(s->side);
  static const bool timing = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  HandleRes r;
  r.device = s->device;
  r.stream = s->stream;
  r.side = s->side;
  r.ev_main = s->ev_main;
  r.ev_side = s->ev_side;
  r.ev_res = s->ev_res;
  for (int k = 0; k < 9; ++k) r.ev[k] = s->ev[k];
  r.hres = s->hres;
  for (int k = 0; k < 2; ++k) {
    r.stage[k] = s->stage[k];
    r.stage_cap[k] = s->stage_cap[k];
  }
  if (r.stream) ResPool::get().give(r);
  HostCache::get().give(s->plan, s->graph);
  const auto t1 = std::chrono::steady_clock::now();
  delete s;
  if (timing)
    std::fprintf(stderr, "[destroy] sync+pool %.2f ms, delete %.2f ms\n",
                 std::chrono::duration<double, std::milli>(t1 - t0).count(),
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count());
}

int dynohip_pool_trim(void) {
  HostCache::get().trim();
  const size_t n = DevPool::get().trim();
  return static_cast<int>(std::min<size_t>(n >> 20, 0x7fffffff));
}

const char* dynohip_last_error(const dynohip_solver* s) { return s ? s->err.c_str() : "null handle"; }

int dynohip_set_graph(dynohip_solver* s, const dynohip_graph_view* g) {
  if (!s || !g) return DYNOHIP_EINVAL;
  const dynohip_factor_block* b[kNTypes] = {&g->pose_to_point, &g->landmark_motion_ternary, &g->between,
                                            &g->prior, &g->landmark_motion_pose, &g->landmark_pose_smoothing};
  for (int t = 0; t < kNTypes; ++t)
    if (b[t]->n && (!b[t]->keys || !b[t]->sigmas || (kMeasDim[t] && !b[t]->measured)))
      return set_err(s, DYNOHIP_EINVAL, "factor type %d: null keys/sigmas/measured", t);
  // copied into the handle's arrays (their capacity is reused across graphs)
  GraphCopy& gc = s->graph;
  // A graph with the current plan's structure (the same factor keys per
  // type, in order) keeps the plan: ordering, schedule and gather lists are
  // functions of the keys alone, and set_values then only refreshes the
  // factor records. Compared exactly (no hash to collide).
  bool same_structure = s->has_graph && s->has_plan && s->nranks == 1;
  for (int t = 0; t < kNTypes && same_structure; ++t)
    same_structure = gc.n[t] == b[t]->n &&
                     std::equal(gc.keys[t].begin(), gc.keys[t].end(), b[t]->keys);
  s->has_graph = false;
  for (int t = 0; t < kNTypes; ++t) {
    const size_t n = b[t]->n;
    gc.n[t] = n;
    if (!same_structure) gc.keys[t].assign(b[t]->keys, b[t]->keys + n * kNKeys[t]);
    if (kMeasDim[t] && n) gc.meas[t].assign(b[t]->measured, b[t]->measured + n * kMeasDim[t]);
    else gc.meas[t].clear();
    gc.sig[t].assign(b[t]->sigmas, b[t]->sigmas + n * kDim[t]);
    if (b[t]->huber_k) gc.hub[t].assign(b[t]->huber_k, b[t]->huber_k + n);
    else gc.hub[t].assign(n, 0.0);
  }
  s->has_graph = true;
  s->lin_valid = false;
  s->has_plan = same_structure;
  s->records_stale = same_structure;
  s->has_values = false;
  s->error_fresh = false;
  return DYNOHIP_OK;
}

// The factor records (indices, measurements, 1/sigma, Huber k: ~40% of a
// plan's bytes) are final once build_plan has laid out the factor types:
// they are staged and copied on a thread of their own while the planner
// builds the rest (same stream; upload_plan's synchronisation covers them).
struct EarlyUpload : PlanHook {
  explicit EarlyUpload(dynohip_solver* h) : s(h) {}
  ~EarlyUpload() override { join(); }
  void types_ready(const Plan& P) override {
    auto body = [this, &P] {
      (void)hipSetDevice(s->device);
      try {
        Uploads up;
        for (int t = 0; t < kNTypes && err == hipSuccess; ++t) {
          const TypePlan& tp = P.types[t];
          if ((err = up.add(s->tb[t].idx, tp.idx)) != hipSuccess || (err = up.add(s->tb[t].meas, tp.meas)) != hipSuccess ||
              (err = up.add(s->tb[t].isig, tp.isig)) != hipSuccess || (err = up.add(s->tb[t].hk, tp.hk)) != hipSuccess)
            break;
        }
        if (err == hipSuccess) err = up.run(s->stage[0], s->stage_cap[0], s->dstage[0], s->stream, false);
      } catch (const std::exception&) {   // host allocation
        err = hipErrorOutOfMemory;
      }
      done = err == hipSuccess;
    };
    // a small plan (PlanCap 1 on the planning thread) copies its few records
    // here: a thread's start, join and first HIP call cost more
    if (PlanPool::cap() == 1) body();
    else th = std::thread(body);
  }
  void join() {
    if (th.joinable()) th.join();
  }
  dynohip_solver* s;
  std::thread th;
  hipError_t err = hipSuccess;
  bool done = false;
};

// The factor records of a kept plan, from the current graph: the same
// checks and the same layout as build_plan's (plan.cpp, factor types).
int refresh_records(dynohip_solver* s) {
  Plan& P = s->plan;
  const GraphCopy& gc = s->graph;
  Uploads up;
  for (int t = 0; t < kNTypes; ++t) {
    TypePlan& tp = P.types[t];
    const size_t n = gc.n[t];
    const std::vector<double>& sig = gc.sig[t];
    const std::vector<double>& meas = gc.meas[t];
    for (size_t i = 0; i < n * kDim[t]; ++i)
      if (!(sig[i] > 0.0 && std::isfinite(sig[i]))) return set_err(s, DYNOHIP_EINVAL, "non-positive sigma");
    for (size_t i = 0; i < n * kMeasDim[t]; ++i)
      if (!std::isfinite(meas[i])) return set_err(s, DYNOHIP_ENONFINITE, "non-finite measurement");
    tp.meas.assign(meas.begin(), meas.end());
    tp.isig.resize(sig.size());
    for (size_t i = 0; i < sig.size(); ++i) tp.isig[i] = 1.0 / sig[i];
    tp.hk.assign(gc.hub[t].begin(), gc.hub[t].end());
    hipError_t e;
    if ((e = up.add(s->tb[t].meas, tp.meas)) != hipSuccess || (e = up.add(s->tb[t].isig, tp.isig)) != hipSuccess ||
        (e = up.add(s->tb[t].hk, tp.hk)) != hipSuccess)
      return set_err(s, DYNOHIP_EHIP, "HIP error %d (%s) in the factor record upload", static_cast<int>(e),
                     hipGetErrorString(e));
  }
  const hipError_t e = up.run(s->stage[0], s->stage_cap[0], s->dstage[0], s->stream, false);
  if (e != hipSuccess)
    return set_err(s, DYNOHIP_EHIP, "HIP error %d (%s) in the factor record upload", static_cast<int>(e),
                   hipGetErrorString(e));
  HIPCHK(s, hipStreamSynchronize(s->stream));   // the staging buffer is reused
  s->records_stale = false;
  s->base_stats_valid = false;
  return DYNOHIP_OK;
}

}  // extern "C"

namespace dynohip {
struct PreparedPlan {
  Plan plan;
};
PreparedPlan* prepare_plan(const dynohip_graph_view& g, const uint64_t* keys, const uint8_t* kind, size_t n, int& rc,
                           std::string& err) {
  auto* p = new PreparedPlan;
  try {
    rc = build_plan(g, keys, kind, n, p->plan, err, 1, 0, true, false, nullptr);
  } catch (const std::exception& ex) {
    rc = DYNOHIP_EINVAL;
    err = std::string("planner: ") + ex.what();
  }
  if (rc == DYNOHIP_OK) return p;
  delete p;
  return nullptr;
}
void free_prepared_plan(PreparedPlan* p) { delete p; }
}  // namespace dynohip

namespace {
int set_values_impl(dynohip_solver* s, const uint64_t* keys, const uint8_t* kind, const double* data, size_t n,
                    Plan* pre);
}

namespace dynohip {
int set_values_prepared(dynohip_solver* s, PreparedPlan* p, const uint64_t* keys, const uint8_t* kind,
                        const double* data, size_t n) {
  return set_values_impl(s, keys, kind, data, n, p ? &p->plan : nullptr);
}
}  // namespace dynohip

namespace {
// pre: a plan built by prepare_plan for this handle's graph and these keys
// (taken instead of planning here; the handle's previous plan goes to *pre)
int set_values_impl(dynohip_solver* s, const uint64_t* keys, const uint8_t* kind, const double* data, size_t n,
                    Plan* pre) {
  if (!s || (n && (!keys || !kind || !data))) return DYNOHIP_EINVAL;
  if (!s->has_graph) return set_err(s, DYNOHIP_ESTATE, "set_graph first");
  (void)hipSetDevice(s->device);
  s->error_fresh = false;
  const bool same = s->has_plan && s->value_keys.size() == n &&
                    std::equal(s->value_keys.begin(), s->value_keys.end(), keys);
  if (!same && pre && s->nranks == 1) {
    // the prepared plan: only its upload is left
    HIPCHK(s, hipStreamSynchronize(s->stream));   // (as below: nothing may still run on the buffers)
    s->has_plan = false;
    std::swap(s->plan, *pre);
    int rc = upload_plan(s, false);
    if (rc) return rc;
    s->value_keys.assign(keys, keys + n);
    s->value_kind.assign(kind, kind + n);
    s->has_plan = true;
    s->records_stale = false;
    ++s->plan_gen;
    s->base_stats_valid = false;
  } else if (!same) {
    const auto tb0 = std::chrono::steady_clock::now();
    // re-planning may grow device buffers, whose old blocks then go to the
    // process-wide pool: nothing of this handle may still run on them (the
    // speculative linearisation of the last try does)
    HIPCHK(s, hipStreamSynchronize(s->stream));
    static const bool sync_timing = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
    if (sync_timing)
      std::fprintf(stderr, "[plan] set_values stream sync      %8.2f ms\n",
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tb0).count());
    s->has_plan = false;
    dynohip_graph_view g = s->graph.view();
    EarlyUpload early(s);
    int rc;
    try {   // nothing thrown crosses the C-ABI (host allocation failures, a planner worker's exception)
      rc = s->nranks > 1 ? build_partitioned_plan(g, keys, kind, n, s->nranks, s->rank, s->plan, s->part,
                                                  s->local_graph, s->err)
                         : build_plan(g, keys, kind, n, s->plan, s->err, 1, 0, true, false, &early);
    } catch (const std::exception& ex) {
      early.join();
      if (early.done) (void)hipStreamSynchronize(s->stream);
      return set_err(s, DYNOHIP_EINVAL, "planner: %s", ex.what());
    }
    early.join();
    if (rc) {
      if (early.done) (void)hipStreamSynchronize(s->stream);   // its staging buffer is reused next time
      return rc;
    }
    if (early.err != hipSuccess) return set_err(s, DYNOHIP_EHIP, "HIP error %d (%s) in the factor record upload",
                                                 static_cast<int>(early.err), hipGetErrorString(early.err));
    static const bool timing = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    if (timing)
      std::fprintf(stderr, "[plan] build_plan (set_values)     %8.2f ms\n",
                   std::chrono::duration<double, std::milli>(t0 - tb0).count());
    rc = upload_plan(s, early.done);
    if (rc) return rc;
    if (timing) {
      (void)hipStreamSynchronize(s->stream);
      std::fprintf(stderr, "[plan] upload                       %8.2f ms\n",
                   std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    if (s->nranks > 1) {
      rc = upload_partition(s);
      if (rc) return rc;
    }
    s->value_keys.assign(keys, keys + n);
    s->value_kind.assign(kind, kind + n);
    s->has_plan = true;
    s->records_stale = false;
    ++s->plan_gen;   // a snapshot of the previous graph's values no longer applies
    s->base_stats_valid = false;
  } else if (s->records_stale) {
    // the plan kept by set_graph: the speculative linearisation of the last
    // try may still read the records being replaced
    HIPCHK(s, hipStreamSynchronize(s->stream));
    const int rc = refresh_records(s);
    if (rc) return rc;
    ++s->plan_gen;
  }
  s->lin_valid = false;
  static const bool vtiming = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
  const auto tv0 = std::chrono::steady_clock::now();
  Plan& P = s->plan;
  std::vector<double> hp(12ull * P.n_pose), hq(3ull * P.n_pt);
  size_t off = 0;
  const bool parted = s->nranks > 1;
  for (size_t i = 0; i < n; ++i) {
    if (kind[i] != s->value_kind[i]) return set_err(s, DYNOHIP_EINVAL, "value kind changed for key %zu", i);
    const int sz = kind[i] == DYNOHIP_POSE3 ? 12 : 3;
    for (int k = 0; k < sz; ++k)
      if (!std::isfinite(data[off + k])) return set_err(s, DYNOHIP_ENONFINITE, "non-finite value");
    const int32_t u = parted ? s->part.local_of[i] : static_cast<int32_t>(i);
    if (u < 0) {  // another rank's landmark
      off += sz;
      continue;
    }
    double* dst = kind[i] == DYNOHIP_POSE3 ? &hp[12ull * P.user_idx[u]] : &hq[3ull * P.user_idx[u]];
    std::memcpy(dst, data + off, sz * sizeof(double));
    off += sz;
  }
  if (!hp.empty()) HIPCHK(s, hipMemcpyAsync(s->pose.p, hp.data(), hp.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
  if (!hq.empty()) HIPCHK(s, hipMemcpyAsync(s->pt.p, hq.data(), hq.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  s->has_values = true;
  const auto tv1 = std::chrono::steady_clock::now();
  const int rc = dynohip_lm_reset(s, &s->prm);
  if (vtiming)
    std::fprintf(stderr, "[values] scatter+upload %.2f ms, initial error %.2f ms\n",
                 std::chrono::duration<double, std::milli>(tv1 - tv0).count(),
                 std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tv1).count());
  return rc;
}
}  // namespace

extern "C" {
int dynohip_set_values(dynohip_solver* s, const uint64_t* keys, const uint8_t* kind, const double* data, size_t n) {
  return set_values_impl(s, keys, kind, data, n, nullptr);
}

int dynohip_get_values(dynohip_solver* s, double* out, size_t n_doubles) {
  int rc = ready(s);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  Plan& P = s->plan;
  std::vector<double> hp(12ull * P.n_pose), hq(3ull * P.n_pt);
  if (!hp.empty()) HIPCHK(s, hipMemcpyAsync(hp.data(), s->pose.p, hp.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
  if (!hq.empty()) HIPCHK(s, hipMemcpyAsync(hq.data(), s->pt.p, hq.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  size_t need = 0;
  for (uint8_t k : s->value_kind) need += k == DYNOHIP_POSE3 ? 12 : 3;
  if (n_doubles < need) return set_err(s, DYNOHIP_EINVAL, "output buffer too small (%zu < %zu)", n_doubles, need);
  size_t off = 0;
  const bool parted = s->nranks > 1;
  for (size_t i = 0; i < s->value_kind.size(); ++i) {
    const int sz = s->value_kind[i] == DYNOHIP_POSE3 ? 12 : 3;
    const int32_t u = parted ? s->part.local_of[i] : static_cast<int32_t>(i);
    if (u < 0) {
      off += sz;
      continue;
    }
    const double* src = s->value_kind[i] == DYNOHIP_POSE3 ? &hp[12ull * P.user_idx[u]] : &hq[3ull * P.user_idx[u]];
    std::memcpy(out + off, src, sz * sizeof(double));
    off += sz;
  }
  return DYNOHIP_OK;
}

int dynohip_graph_error(dynohip_solver* s, double* error_out) {
  int rc = ready(s);
  if (rc) return rc;
  if (!error_out) return DYNOHIP_EINVAL;
  (void)hipSetDevice(s->device);
  return compute_error(s, s->pose.p, s->pt.p, error_out);
}

int dynohip_lm_reset(dynohip_solver* s, const dynohip_lm_params* p) {
  int rc = ready(s);
  if (rc) return rc;
  if (!p) return DYNOHIP_EINVAL;
  if (p->diagonal_damping || !p->use_fixed_lambda_factor)
    return set_err(s, DYNOHIP_EINVAL, "only diagonalDamping=false, useFixedLambdaFactor=true are supported");
  (void)hipSetDevice(s->device);
  s->prm = *p;
  s->lin_valid = false;
  s->lambda = p->lambda_initial;
  s->iterations = 0;
  s->inner = 0;
  s->converged = 0;
  s->trace.clear();
  s->n_lin = 0;
  s->n_solves = 0;
  for (double& v : s->phase_ms) v = 0.0;
  if (s->error_fresh) return DYNOHIP_OK;
  rc = compute_error(s, s->pose.p, s->pt.p, &s->error);
  s->error_fresh = rc == 0;
  return rc;
}

int dynohip_iterate(dynohip_solver* s, dynohip_lm_summary* out) {
  int rc = ready(s);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  const double e0 = s->error;
  rc = lm_iterate(s);
  if (rc) return rc;
  fill_summary(s, e0, out);
  return DYNOHIP_OK;
}

// NonlinearOptimizer::defaultOptimize + checkConvergence
int dynohip_optimize(dynohip_solver* s, const dynohip_lm_params* p, dynohip_lm_summary* out) {
  int rc = dynohip_lm_reset(s, p);
  if (rc) return rc;
  const double initial = s->error;
  double currentError = s->error;
  if (currentError <= p->error_tol || s->iterations >= p->max_iterations) {
    s->converged = currentError <= p->error_tol;
    fill_summary(s, initial, out);
    return DYNOHIP_OK;
  }
  double newError = currentError;
  do {
    currentError = newError;
    rc = lm_iterate(s);
    if (rc) return rc;
    newError = s->error;
    bool conv;
    if (newError <= p->error_tol) {
      conv = true;
    } else {
      const double absd = currentError - newError;
      const double reld = absd / currentError;
      conv = (reld <= p->relative_error_tol) || (absd <= p->absolute_error_tol);
    }
    s->converged = conv;
  } while (s->iterations < p->max_iterations && !s->converged && std::isfinite(currentError));
  fill_summary(s, initial, out);
  return DYNOHIP_OK;
}

int dynohip_get_trace(dynohip_solver* s, dynohip_trace_entry* out, size_t capacity, size_t* n_out) {
  if (!s) return DYNOHIP_EINVAL;
  const size_t n = std::min(capacity, s->trace.size());
  if (out && n) std::memcpy(out, s->trace.data(), n * sizeof(dynohip_trace_entry));
  if (n_out) *n_out = s->trace.size();
  return DYNOHIP_OK;
}

size_t dynohip_linearize_size(const dynohip_solver* s) {
  if (!s || !s->has_plan) return 0;
  size_t n = 0;
  for (int t = 0; t < kNTypes; ++t) n += static_cast<size_t>(s->plan.types[t].n) * kDim[t] * (kCols[t] + 1);
  return n;
}

int dynohip_linearize(dynohip_solver* s, double* out, size_t n_doubles) {
  int rc = ready(s);
  if (rc) return rc;
  if (n_doubles < dynohip_linearize_size(s)) return set_err(s, DYNOHIP_EINVAL, "output buffer too small");
  (void)hipSetDevice(s->device);
  s->lin_valid = false;
  if (int rc2 = enqueue_linearize(s, s->pose.p, s->pt.p, nullptr, true)) return rc2;
  const Plan& P = s->plan;
  std::vector<double> rec;
  size_t o = 0;
  for (int t = 0; t < kNTypes; ++t) {
    const TypePlan& tp = P.types[t];
    if (tp.n == 0) continue;
    rec.resize(static_cast<size_t>(tp.stride) * tp.n);
    HIPCHK(s, hipMemcpyAsync(rec.data(), s->arena.p + tp.base, rec.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(s, hipStreamSynchronize(s->stream));
    const int d = kDim[t];
    for (int i = 0; i < tp.n; ++i) {
      const double* r = rec.data() + static_cast<size_t>(tp.stride) * i;
      for (int k = 0; k < d; ++k) {
        for (int sl = 0; sl < kNKeys[t]; ++sl) {
          const int ds = kSlotKind[t][sl] == 0 ? 6 : 3;
          const double* blk = r + d * kColStart[t][sl];
          for (int c = 0; c < ds; ++c) out[o++] = blk[k * ds + c];
        }
        out[o++] = r[d * kCols[t] + k];
      }
    }
  }
  return DYNOHIP_OK;
}

int dynohip_solve_delta(dynohip_solver* s, double lambda, double* delta_out, size_t n_doubles, int* solved_out) {
  int rc = ready(s);
  if (rc) return rc;
  if (s->nranks > 1) return set_err(s, DYNOHIP_EINVAL, "solve_delta: single-GPU handles only");
  if (!(lambda >= 0.0) || !std::isfinite(lambda)) return set_err(s, DYNOHIP_EINVAL, "solve_delta: lambda %g", lambda);
  size_t need = 0;
  for (uint8_t k : s->value_kind) need += k == DYNOHIP_POSE3 ? 6 : 3;
  if (!delta_out || n_doubles < need)
    return set_err(s, DYNOHIP_EINVAL, "solve_delta: output buffer too small (%zu < %zu)", n_doubles, need);
  (void)hipSetDevice(s->device);
  const Plan& P = s->plan;
  // the same launches as one tryLambda of lm_iterate, at the current values
  s->lin_valid = false;
  rc = enqueue_linearize(s, s->pose.p, s->pt.p, s->result.p + 2);
  if (rc) return rc;
  rc = enqueue_try(s, lambda);
  if (rc) return rc;
  const size_t nrp = static_cast<size_t>(P.NT) * kTile;
  std::vector<double> hx(6ull * P.n_pose), hq(3ull * P.n_pt);
  double res[5];
  if (!hx.empty()) HIPCHK(s, hipMemcpyAsync(hx.data(), s->xy.p + nrp, hx.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
  if (!hq.empty()) HIPCHK(s, hipMemcpyAsync(hq.data(), s->dpt.p, hq.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipMemcpyAsync(res, s->result.p, sizeof(res), hipMemcpyDeviceToHost, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  int fail = 0;
  std::memcpy(&fail, &res[4], sizeof(int));
  if (fail & 6) return set_err(s, DYNOHIP_EHIP, "solve_delta: dependency wait timed out");
  if (solved_out) *solved_out = fail == 0 && std::isfinite(res[0]);
  size_t off = 0;
  for (size_t i = 0; i < s->value_kind.size(); ++i) {
    const bool pose = s->value_kind[i] == DYNOHIP_POSE3;
    const int sz = pose ? 6 : 3;
    const double* src = pose ? &hx[6ull * P.user_idx[i]] : &hq[3ull * P.user_idx[i]];
    std::memcpy(delta_out + off, src, sz * sizeof(double));
    off += sz;
  }
  return DYNOHIP_OK;
}

int dynohip_values_snapshot(dynohip_solver* s) {
  int rc = ready(s);
  if (rc) return rc;
  (void)hipSetDevice(s->device);
  const Plan& P = s->plan;
  // sized for the current plan (a re-planned handle may hold a larger graph);
  // a grown buffer's old block goes to the pool with the stream idle
  HIPCHK(s, hipStreamSynchronize(s->stream));
  if (P.n_pose) HIPCHK(s, s->pose_snap.alloc(12ull * P.n_pose));
  if (P.n_pt) HIPCHK(s, s->pt_snap.alloc(3ull * P.n_pt));
  if (P.n_pose) HIPCHK(s, hipMemcpyAsync(s->pose_snap.p, s->pose.p, 12ull * P.n_pose * sizeof(double), hipMemcpyDeviceToDevice, s->stream));
  if (P.n_pt) HIPCHK(s, hipMemcpyAsync(s->pt_snap.p, s->pt.p, 3ull * P.n_pt * sizeof(double), hipMemcpyDeviceToDevice, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  s->snap_gen = s->plan_gen;
  return DYNOHIP_OK;
}

int dynohip_values_restore(dynohip_solver* s) {
  int rc = ready(s);
  if (rc) return rc;
  const Plan& P = s->plan;
  // a snapshot taken before the last re-plan belongs to another graph, even
  // when its buffer sizes happen to match (equal-length sliding windows)
  if (s->snap_gen == 0 || s->snap_gen != s->plan_gen)
    return set_err(s, DYNOHIP_ESTATE, "no snapshot of the current graph's values");
  (void)hipSetDevice(s->device);
  s->lin_valid = false;
  s->error_fresh = false;
  if (P.n_pose) HIPCHK(s, hipMemcpyAsync(s->pose.p, s->pose_snap.p, 12ull * P.n_pose * sizeof(double), hipMemcpyDeviceToDevice, s->stream));
  if (P.n_pt) HIPCHK(s, hipMemcpyAsync(s->pt.p, s->pt_snap.p, 3ull * P.n_pt * sizeof(double), hipMemcpyDeviceToDevice, s->stream));
  HIPCHK(s, hipStreamSynchronize(s->stream));
  return DYNOHIP_OK;
}

int dynohip_get_stats(dynohip_solver* s, dynohip_stats* out) {
  if (!s || !out) return DYNOHIP_EINVAL;
  if (s->has_plan && !s->base_stats_valid) {
    compute_base_stats(s);
    s->base_stats_valid = true;
  }
  *out = s->base_stats;
  out->ms_linearize = s->phase_ms[0];
  out->ms_schur = s->phase_ms[1];
  out->ms_assembly = s->phase_ms[2];
  out->ms_cholesky = s->phase_ms[3];
  out->ms_solve = s->phase_ms[4];
  out->ms_backsub = s->phase_ms[5];
  out->ms_retract_error = s->phase_ms[6];
  out->n_linearize = s->n_lin;
  out->n_solves = s->n_solves;
  return DYNOHIP_OK;
}

int dynohip_set_exec_options(dynohip_solver* s, int wide_updates, int level_backward, int level_factor) {
  if (!s || wide_updates < 0) return DYNOHIP_EINVAL;
  s->sd.wide_updates = wide_updates;
  s->sd.level_backward = level_backward != 0;
  s->sd.persistent_factor = level_factor == 0;
  if (!s->sd.persistent_factor && !s->side) {
    (void)hipSetDevice(s->device);
    if (hipStreamCreateWithFlags(&s->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev_side, hipEventDisableTiming) != hipSuccess)
      return set_err(s, DYNOHIP_EHIP, "second stream");
  }
  return DYNOHIP_OK;
}

int dynohip_set_partition(dynohip_solver* s, int nranks, int rank, dynohip_allreduce_fn allreduce, void* ctx) {
  if (!s || nranks < 1 || rank < 0 || rank >= nranks) return DYNOHIP_EINVAL;
  if (nranks > 1 && ((nranks & (nranks - 1)) != 0 || !allreduce))
    return set_err(s, DYNOHIP_EINVAL, "partitioned solve needs a power-of-two rank count and an all-reduce");
  s->nranks = nranks;
  s->rank = rank;
  s->comm = allreduce;
  s->comm_ctx = ctx;
  s->has_plan = false;
  s->has_values = false;
  s->lin_valid = false;
  s->error_fresh = false;
  return DYNOHIP_OK;
}

int dynohip_value_owner(dynohip_solver* s, int32_t* owner_out, size_t n, int64_t* exchange_doubles) {
  int rc = ready(s);
  if (rc) return rc;
  if (n != s->value_kind.size() || (n && !owner_out)) return set_err(s, DYNOHIP_EINVAL, "owner buffer size");
  for (size_t i = 0; i < n; ++i) owner_out[i] = s->nranks > 1 ? s->part.value_owner[i] : 0;
  if (exchange_doubles) *exchange_doubles = s->nranks > 1 ? s->xtotal : 0;
  return DYNOHIP_OK;
}

int dynohip_set_timing(dynohip_solver* s, int enabled) {
  if (!s) return DYNOHIP_EINVAL;
  s->timing = enabled != 0;
  return DYNOHIP_OK;
}

}  // extern "C"
