#include <chrono>
#include <cstdio>
#include <cstdlib>
// plan.cpp — factor graph -> device layout / gather lists (see plan.hpp).
#include "plan.hpp"
#include "plan_pool.hpp"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <unistd.h>

#include <atomic>
#include <future>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <unordered_map>

namespace dynohip {

namespace {

struct PoseSortKey {
  uint64_t frame;
  unsigned chr, label;
  uint64_t key;
  int32_t user;
};

// frame order of a pose key: X(k) -> k; LabeledSymbol H/L(j,k) -> k
// (BackendDefinitions.hpp:57-88)
PoseSortKey pose_sort_key(uint64_t key, int32_t user) {
  PoseSortKey s;
  s.key = key;
  s.user = user;
  s.chr = static_cast<unsigned>(key >> 56);
  const unsigned l = static_cast<unsigned>((key >> 48) & 0xff);
  if (s.chr > 0 && l > 0) {
    s.label = l;
    s.frame = key & ((1ULL << 48) - 1);
  } else {
    s.label = 0;
    s.frame = key & ((1ULL << 56) - 1);
  }
  return s;
}

uint32_t block_off(const TypePlan& tp, int type, int i, int slot) {
  return static_cast<uint32_t>(tp.base + static_cast<uint64_t>(tp.stride) * i +
                               static_cast<uint64_t>(kDim[type]) * kColStart[type][slot]);
}
uint32_t b_off(const TypePlan& tp, int type, int i) {
  return static_cast<uint32_t>(tp.base + static_cast<uint64_t>(tp.stride) * i +
                               static_cast<uint64_t>(kDim[type]) * kCols[type]);
}

// build a CSR gather list from (target, entry) pairs, stable in generation order
constexpr int pose_slots(int t) {
  int n = 0;
  for (int s = 0; s < 4; ++s) n += kSlotKind[t][s] == 0;
  return n;
}
constexpr int kNPoseSlots[kNTypes] = {pose_slots(0), pose_slots(1), pose_slots(2), pose_slots(3), pose_slots(4),
                                      pose_slots(5)};

// open-addressing key -> index table (linear probing, power-of-two size);
// replaces std::unordered_map on the hot key lookups of planning
class KeyIndex {
 public:
  // storage: vectors owned by the caller (Plan::Scratch), refilled here
  KeyIndex(size_t n, std::vector<uint64_t>& keys, std::vector<int32_t>& vals) : keys_(keys), vals_(vals) {
    size_t cap = 16;
    while (cap < 2 * n + 1) cap <<= 1;
    mask_ = cap - 1;
    keys_.assign(cap, 0);
    vals_.assign(cap, -1);
  }
  // false if the key is already present
  bool insert(uint64_t key, int32_t v) {
    size_t h = hash(key);
    while (vals_[h] >= 0) {
      if (keys_[h] == key) return false;
      h = (h + 1) & mask_;
    }
    keys_[h] = key;
    vals_[h] = v;
    return true;
  }
  int32_t find(uint64_t key) const {
    size_t h = hash(key);
    while (vals_[h] >= 0) {
      if (keys_[h] == key) return vals_[h];
      h = (h + 1) & mask_;
    }
    return -1;
  }

 private:
  size_t hash(uint64_t k) const { return static_cast<size_t>((k * 0x9E3779B97F4A7C15ull) >> 17) & mask_; }
  size_t mask_;
  std::vector<uint64_t>& keys_;
  std::vector<int32_t>& vals_;
};

// CSR by target ranges: worker r owns the targets [tcut[r], tcut[r+1]) and
// runs the enumeration emit(r, fn) itself, keeping only its own targets (the
// emitter may skip what it knows lies outside range r). Every target keeps
// the enumeration order of its entries, so the lists equal a single-threaded
// two-pass build, and each worker fills one contiguous part of the output:
// cache-local writes instead of one scatter over the whole list.
template <typename Emit>
void csr_target_ranges(size_t ntargets, const std::vector<int64_t>& tcut, Emit&& emit, GatherList& out) {
  const int nr = static_cast<int>(tcut.size()) - 1;
  auto parallel = [&](auto&& body) { PlanPool::get().run(nr, body); };
  auto T0 = std::chrono::steady_clock::now();
  out.start.assign(ntargets + 1, 0);
  parallel([&](int r) {
    const int64_t t0 = tcut[r], t1 = tcut[r + 1];
    emit(r, [&](int64_t t, const GEntry&) {
      if (t >= t0 && t < t1) out.start[t + 1]++;
    });
  });
  auto T1 = std::chrono::steady_clock::now();
  for (size_t t = 0; t < ntargets; ++t) out.start[t + 1] += out.start[t];
  out.ent.resize(out.start[ntargets]);
  auto T2 = std::chrono::steady_clock::now();
  parallel([&](int r) {
    const int64_t t0 = tcut[r], t1 = tcut[r + 1];
    std::vector<int64_t> cur(out.start.begin() + t0, out.start.begin() + t1);
    emit(r, [&](int64_t t, const GEntry& e) {
      if (t >= t0 && t < t1) out.ent[cur[t - t0]++] = e;
    });
  });
  auto T3 = std::chrono::steady_clock::now();
  if (std::getenv("DYNOHIP_PLAN_TIMING"))
    std::fprintf(stderr, "  csr nt=%zu nw=%d ent=%zu count %.2f alloc %.2f fill %.2f ms\n", ntargets, nr, out.ent.size(),
                 std::chrono::duration<double, std::milli>(T1 - T0).count(),
                 std::chrono::duration<double, std::milli>(T2 - T1).count(),
                 std::chrono::duration<double, std::milli>(T3 - T2).count());
}


// even cut of [0, n) targets into the planner's workers, one per 1024
// targets at most (a sliding window's few hundred targets take one: each
// worker of a target-range CSR enumerates every source, so a small graph
// paid the pool dispatch for nothing — window planning 6.2 -> 2.6 ms here)
std::vector<int64_t> even_cuts(int64_t n) {
  const int nw = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(PlanPool::get().workers(), n / 1024 + 1)));
  std::vector<int64_t> c(nw + 1);
  for (int r = 0; r <= nw; ++r) c[r] = n * r / nw;
  return c;
}

}  // namespace

// values + factors below which a plan runs its parallel sections on one
// thread (a C2-stream window: ~1.5k values, ~4k factors; C2: 185k).
// DYNOHIP_SMALL_PLAN_ITEMS overrides it (0: no small-plan cap), so the tests
// can compare a capped plan with the threaded one (tests/test_plan_digest.py)
static size_t small_plan_items() {
  static const size_t v = [] {
    const char* e = std::getenv("DYNOHIP_SMALL_PLAN_ITEMS");
    return e ? static_cast<size_t>(std::strtoull(e, nullptr, 10)) : size_t{20000};
  }();
  return v;
}

static double plan_now() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void plan_mark(const char* what, double& t) {
  static const bool on = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
  const double n = plan_now();
  if (on) std::fprintf(stderr, "[plan] %-28s %8.2f ms\n", what, n - t);
  t = n;
}

void compute_red_slots(Plan& P) {
  const int64_t nt = static_cast<int64_t>(P.red_A.size());
  P.red_slot.resize(4 * static_cast<size_t>(nt));
  auto lookup = [&](int i, int j) -> uint32_t {   // stored tile of natural tiles (i, j), as tile_index
    uint32_t tr = 0;
    if (P.tile_pos[i] < P.tile_pos[j]) { std::swap(i, j); tr = 1u << 31; }
    const auto b = P.row_col.begin() + P.row_start[i], e = P.row_col.begin() + P.row_start[i + 1];
    const auto it = std::lower_bound(b, e, j);
    if (it == e || *it != j) return ~0u;
    return static_cast<uint32_t>(P.row_slot[it - P.row_col.begin()]) | tr;
  };
  parallel_for(nt, [&](int64_t t0, int64_t t1) {
    for (int64_t t = t0; t < t1; ++t) {
      const int r0 = 6 * P.red_A[t] / kTile, r1 = (6 * P.red_A[t] + 5) / kTile;
      const int c0 = 6 * P.red_B[t] / kTile, c1 = (6 * P.red_B[t] + 5) / kTile;
      uint32_t* o = P.red_slot.data() + 4 * t;
      o[0] = lookup(r0, c0);
      o[1] = c1 != c0 ? lookup(r0, c1) : ~0u;
      o[2] = r1 != r0 ? lookup(r1, c0) : ~0u;
      o[3] = (r1 != r0 && c1 != c0) ? lookup(r1, c1) : ~0u;
    }
  });
  // targets by entry count (class c holds the targets of <= 4 << c entries;
  // the last class all larger ones), each class in target order
  const int64_t* st = P.gRed.start.data();
  auto cls = [&](int64_t t) {
    const int64_t m = st[t + 1] - st[t];
    int c = 0;
    while (c < Plan::kRedClasses - 1 && m > (int64_t{4} << c)) ++c;
    return c;
  };
  int32_t pos[Plan::kRedClasses + 1] = {};
  for (int c = 0; c < Plan::kRedClasses; ++c) P.red_ncls[c] = 0;
  if (P.gRed.start.size() != static_cast<size_t>(nt) + 1) {   // no band gather (structure-only plans)
    P.red_order.clear();
    P.red_blocks.clear();
    return;
  }
  for (int64_t t = 0; t < nt; ++t) ++P.red_ncls[cls(t)];
  for (int c = 0; c < Plan::kRedClasses; ++c) pos[c + 1] = pos[c] + P.red_ncls[c];
  P.red_order.resize(static_cast<size_t>(nt));
  for (int64_t t = 0; t < nt; ++t) P.red_order[pos[cls(t)]++] = static_cast<int32_t>(t);
  // The band blocks by column. Every class spans every column (a column's
  // targets near the diagonal have the most entries, the far ones the
  // fewest), so class after class each pass streamed the chains' W and Y
  // blocks again (NS: 2.4x the deduplicated operand bytes from HBM). In
  // column order the classes' blocks of one column band run together, on
  // one XCD (xcd_block), and share those operands in its L2.
  struct Blk {
    int32_t col, cls, k;
  };
  std::vector<Blk> blks;
  int32_t off = 0;
  for (int c = 0; c < Plan::kRedClasses; ++c) {
    const int lanes = c < Plan::kRedClasses - 1 ? 8 << c : 128;
    const int per = kRedBlock / lanes;   // targets per block
    for (int32_t k = 0; k * per < P.red_ncls[c]; ++k)
      blks.push_back(Blk{P.red_B[P.red_order[off + k * per]], c, k});
    off += P.red_ncls[c];
  }
  // (larger classes first within a column: their targets hold the longest entry chains)
  std::stable_sort(blks.begin(), blks.end(), [](const Blk& a, const Blk& b) {
    return a.col < b.col || (a.col == b.col && a.cls > b.cls);
  });
  P.red_blocks.resize(blks.size());
  for (size_t i = 0; i < blks.size(); ++i) P.red_blocks[i] = (blks[i].k << 3) | blks[i].cls;
}

void plan_recycle(Plan& P) {
  Plan f;
  // every array: cleared (size 0, capacity kept) and moved into the fresh plan
  auto k = [](auto& dst, auto& src) {
    src.clear();
    dst.swap(src);
  };
  k(f.user_kind, P.user_kind); k(f.user_idx, P.user_idx); k(f.pose_key, P.pose_key); k(f.pt_key, P.pt_key);
  k(f.comp_start, P.comp_start); k(f.comp_nb_start, P.comp_nb_start); k(f.nb_pose, P.nb_pose);
  k(f.nb_comp, P.nb_comp); k(f.comp_y_base, P.comp_y_base); k(f.nbedge_start, P.nbedge_start);
  k(f.nbedge_pt, P.nbedge_pt); k(f.nbedge_w, P.nbedge_w);
  k(f.edge_pt, P.edge_pt); k(f.edge_pose, P.edge_pose); k(f.pt_edge_start, P.pt_edge_start);
  for (int t = 0; t < kNTypes; ++t) {
    k(f.types[t].idx, P.types[t].idx); k(f.types[t].meas, P.types[t].meas);
    k(f.types[t].isig, P.types[t].isig); k(f.types[t].hk, P.types[t].hk);
  }
  GatherList Plan::*gl[] = {&Plan::gD, &Plan::gE, &Plan::gGp, &Plan::gW, &Plan::gRed, &Plan::gGred};
  for (auto m : gl) {
    k((f.*m).start, (P.*m).start);
    k((f.*m).ent, (P.*m).ent);
  }
  k(f.red_A, P.red_A); k(f.red_B, P.red_B); k(f.red_slot, P.red_slot); k(f.red_order, P.red_order);
  k(f.red_blocks, P.red_blocks);
  k(f.lgroup, P.lgroup); k(f.lone_pose, P.lone_pose); k(f.lone_blk, P.lone_blk); k(f.lin_list0, P.lin_list0);
  k(f.band_D, P.band_D); k(f.tile_pos, P.tile_pos); k(f.row_start, P.row_start); k(f.row_col, P.row_col);
  k(f.row_slot, P.row_slot); k(f.ftask, P.ftask); k(f.pairs, P.pairs); k(f.flevel, P.flevel);
  k(f.fpanels, P.fpanels); k(f.fdep_start, P.fdep_start); k(f.fdep, P.fdep); k(f.fqueue, P.fqueue);
  k(f.btask, P.btask); k(f.blevel, P.blevel); k(f.bent, P.bent); k(f.bpart, P.bpart); k(f.bplevel, P.bplevel);
  k(f.tile_owner, P.tile_owner); k(f.sep_nodes, P.sep_nodes); k(f.phases, P.phases);
  k(f.rhs0_tile, P.rhs0_tile); k(f.rhs0_start, P.rhs0_start); k(f.rhs0_slot, P.rhs0_slot);
  f.scratch = std::move(P.scratch);   // contents are refilled by build_plan
  P = std::move(f);
}

int build_plan(const dynohip_graph_view& g, const uint64_t* keys, const uint8_t* kind, size_t n, Plan& P,
               std::string& err, int nranks, int rank, bool with_schedule, bool structure_only, PlanHook* hook) {
  double tmark = plan_now();
  // small graphs plan on this thread (and its schedule thread) alone
  const size_t n_fac = g.pose_to_point.n + g.landmark_motion_ternary.n + g.between.n + g.prior.n +
                       g.landmark_motion_pose.n + g.landmark_pose_smoothing.n;
  const int pcap = n + n_fac < small_plan_items() ? 1 : 0;
  PlanCap plan_cap(pcap);
  plan_recycle(P);
  P.nranks = nranks;
  P.rank = rank;
  // ---- values: key lookup ----
  Plan::Scratch& sc = P.scratch;
  KeyIndex key_to_user(n, sc.key_k, sc.key_v);
  for (size_t i = 0; i < n; ++i) {
    if (kind[i] > 1) { err = "bad value kind"; return DYNOHIP_EINVAL; }
    if (!key_to_user.insert(keys[i], static_cast<int32_t>(i))) { err = "duplicate value key"; return DYNOHIP_EINVAL; }
  }
  P.user_kind.assign(kind, kind + n);
  P.user_idx.assign(n, -1);
  plan_mark("value key index", tmark);

  const dynohip_factor_block* blocks[kNTypes] = {&g.pose_to_point, &g.landmark_motion_ternary, &g.between,
                                                 &g.prior, &g.landmark_motion_pose, &g.landmark_pose_smoothing};
  // user index per factor slot
  auto& fuser = sc.fuser;   // user index per factor slot (every entry written below)
  for (int t = 0; t < kNTypes; ++t) {
    const auto* b = blocks[t];
    if (b->n == 0) continue;
    if (!b->keys || !b->sigmas || (kMeasDim[t] > 0 && !b->measured)) {
      err = "factor type " + std::to_string(t) + ": null keys/sigmas/measured";
      return DYNOHIP_EINVAL;
    }
    fuser[t].resize(b->n * kNKeys[t]);
    // fast path on the workers; any failure is re-found below, in order, for its message
    // (bad[0]: a key; bad[1]: a sigma; bad[2]: a measurement)
    std::vector<uint8_t> bad(3, 0);
    parallel_for(static_cast<int64_t>(b->n), [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; ++i)
        for (int s = 0; s < kNKeys[t]; ++s) {
          const int32_t u = key_to_user.find(b->keys[i * kNKeys[t] + s]);
          const int want = kSlotKind[t][s] == 0 ? DYNOHIP_POSE3 : DYNOHIP_POINT3;
          if (u < 0 || kind[u] != want) {
            __atomic_store_n(&bad[0], 1, __ATOMIC_RELAXED);
            return;
          }
          fuser[t][i * kNKeys[t] + s] = u;
        }
      bool sig_ok = true, meas_ok = true;
      for (int64_t i = i0 * kDim[t]; i < i1 * kDim[t]; ++i)
        sig_ok &= b->sigmas[i] > 0.0 && std::isfinite(b->sigmas[i]);
      for (int64_t i = i0 * kMeasDim[t]; i < i1 * kMeasDim[t]; ++i) meas_ok &= std::isfinite(b->measured[i]) != 0;
      if (!sig_ok) __atomic_store_n(&bad[1], 1, __ATOMIC_RELAXED);
      if (!meas_ok) __atomic_store_n(&bad[2], 1, __ATOMIC_RELAXED);
    });
    if (bad[0])
    for (size_t i = 0; i < b->n; ++i)
      for (int s = 0; s < kNKeys[t]; ++s) {
        const uint64_t key = b->keys[i * kNKeys[t] + s];
        const int32_t u = key_to_user.find(key);
        if (u < 0) {
          err = "factor type " + std::to_string(t) + " #" + std::to_string(i) + ": key " + std::to_string(key) +
                " does not exist in the values";
          return DYNOHIP_EKEY;
        }
        const int want = kSlotKind[t][s] == 0 ? DYNOHIP_POSE3 : DYNOHIP_POINT3;
        if (kind[u] != want) {
          err = "factor type " + std::to_string(t) + " #" + std::to_string(i) + ": key has wrong value kind";
          return DYNOHIP_EINVAL;
        }
        fuser[t][i * kNKeys[t] + s] = u;
      }
    if (bad[1]) { err = "non-positive sigma"; return DYNOHIP_EINVAL; }
    if (bad[2]) { err = "non-finite measurement"; return DYNOHIP_ENONFINITE; }
  }

  plan_mark("before poses: frame order", tmark);
  // ---- poses: frame order ----
  {
    std::vector<PoseSortKey> ps;
    for (size_t i = 0; i < n; ++i)
      if (kind[i] == DYNOHIP_POSE3) ps.push_back(pose_sort_key(keys[i], static_cast<int32_t>(i)));
    std::sort(ps.begin(), ps.end(), [](const PoseSortKey& a, const PoseSortKey& b) {
      if (a.frame != b.frame) return a.frame < b.frame;
      if (a.chr != b.chr) return a.chr < b.chr;
      if (a.label != b.label) return a.label < b.label;
      return a.key < b.key;
    });
    P.n_pose = static_cast<int>(ps.size());
    P.pose_key.resize(ps.size());
    for (size_t r = 0; r < ps.size(); ++r) {
      P.user_idx[ps[r].user] = static_cast<int32_t>(r);
      P.pose_key[r] = ps[r].key;
    }
  }

  plan_mark("before point chains", tmark);
  // ---- point chains ----
  // adjacency between points from factors with two point slots: at most two
  // distinct neighbours per point (a chain), held flat
  std::vector<int32_t>& adj = sc.adj;
  adj.assign(2 * n, -1);
  std::vector<uint8_t> deg(n, 0);
  bool too_many = false;
  auto link = [&](int32_t a, int32_t b) {
    if (adj[2 * a] == b || adj[2 * a + 1] == b) return;
    if (deg[a] == 2) { too_many = true; return; }
    adj[2 * a + deg[a]++] = b;
  };
  for (int t = 0; t < kNTypes; ++t) {
    const int nk = kNKeys[t];
    int ps[4], np = 0;
    for (int s = 0; s < nk; ++s)
      if (kSlotKind[t][s] == 1) ps[np++] = s;
    if (np < 2) continue;
    if (np > 2) { err = "factor with >2 point slots unsupported"; return DYNOHIP_ESTRUCT; }
    for (size_t i = 0; i < blocks[t]->n; ++i) {
      const int32_t a = fuser[t][i * nk + ps[0]], b = fuser[t][i * nk + ps[1]];
      if (a == b) { err = "factor links a point to itself"; return DYNOHIP_ESTRUCT; }
      link(a, b);
      link(b, a);
    }
  }
  if (too_many) { err = "point component is not a chain (degree > 2)"; return DYNOHIP_ESTRUCT; }
  {
    std::vector<char> seen(n, 0);
    // chains in walk order from the endpoint with the smallest key, flat
    std::vector<int32_t> walks, wstart{0}, comp;
    walks.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      if (kind[i] != DYNOHIP_POINT3 || seen[i]) continue;
      seen[i] = 1;
      if (deg[i] == 0) {   // a lone point (every static landmark)
        walks.push_back(static_cast<int32_t>(i));
        wstart.push_back(static_cast<int32_t>(walks.size()));
        continue;
      }
      // collect the component
      comp.assign(1, static_cast<int32_t>(i));
      size_t nedges2 = 0;
      for (size_t q = 0; q < comp.size(); ++q) {
        const int32_t u = comp[q];
        nedges2 += deg[u];
        for (int k = 0; k < deg[u]; ++k) {
          const int32_t w = adj[2 * u + k];
          if (!seen[w]) { seen[w] = 1; comp.push_back(w); }
        }
      }
      if (nedges2 / 2 != comp.size() - 1) { err = "point component is not a chain (cycle)"; return DYNOHIP_ESTRUCT; }
      int32_t start = -1;
      for (int32_t u : comp)
        if (deg[u] <= 1 && (start < 0 || keys[u] < keys[start])) start = u;
      int32_t prev = -1, cur = start;
      for (size_t q = 0; q < comp.size(); ++q) {
        walks.push_back(cur);
        int32_t nxt = -1;
        for (int k = 0; k < deg[cur]; ++k)
          if (adj[2 * cur + k] != prev) nxt = adj[2 * cur + k];
        prev = cur;
        cur = nxt;
      }
      wstart.push_back(static_cast<int32_t>(walks.size()));
    }
    // longest chains first (stable, a counting sort by length): the chain
    // kernels run a thread per chain, so a wave then holds chains of one
    // length and the long ones start first
    const int nchains = static_cast<int>(wstart.size()) - 1;
    int maxlen = 0;
    for (int c = 0; c < nchains; ++c) maxlen = std::max(maxlen, wstart[c + 1] - wstart[c]);
    std::vector<int32_t> lcnt(static_cast<size_t>(maxlen) + 2, 0);
    for (int c = 0; c < nchains; ++c) lcnt[maxlen - (wstart[c + 1] - wstart[c]) + 1]++;
    for (int L = 0; L <= maxlen; ++L) lcnt[L + 1] += lcnt[L];
    std::vector<int32_t> order(nchains);
    for (int c = 0; c < nchains; ++c) order[lcnt[maxlen - (wstart[c + 1] - wstart[c])]++] = c;
    int32_t next_pt = 0;
    P.comp_start.reserve(nchains + 1);
    P.pt_key.reserve(walks.size());
    P.comp_start.push_back(0);
    for (int c : order) {
      for (int32_t q = wstart[c]; q < wstart[c + 1]; ++q) {
        const int32_t u = walks[q];
        P.user_idx[u] = next_pt++;
        P.pt_key.push_back(keys[u]);
      }
      P.comp_start.push_back(next_pt);
    }
    P.max_chain = maxlen;
    P.n_pt = next_pt;
    P.n_comp = static_cast<int>(P.comp_start.size()) - 1;
  }
  std::vector<int32_t> comp_of(P.n_pt);
  for (int c = 0; c < P.n_comp; ++c)
    for (int32_t i = P.comp_start[c]; i < P.comp_start[c + 1]; ++i) comp_of[i] = c;

  plan_mark("before factor types: indices, measurements, arena records", tmark);
  // ---- factor types: indices, measurements, arena records ----
  uint64_t arena = 0;
  for (int t = 0; t < kNTypes; ++t) {
    TypePlan& tp = P.types[t];
    const auto* b = blocks[t];
    tp.n = static_cast<int>(b->n);
    tp.stride = static_cast<uint32_t>((kDim[t] * (kCols[t] + 1) + 1) & ~1);
    tp.base = arena;
    arena += static_cast<uint64_t>(tp.stride) * tp.n;
    // uninitialised, then filled (copies included) on the workers
    tp.idx.resize(b->n * kNKeys[t]);
    tp.meas.resize(b->measured ? b->n * kMeasDim[t] : 0);
    tp.isig.resize(b->n * kDim[t]);
    tp.hk.resize(b->n);
    parallel_for(static_cast<int64_t>(b->n), [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0 * kNKeys[t]; i < i1 * kNKeys[t]; ++i) tp.idx[i] = P.user_idx[fuser[t][i]];
      for (int64_t i = i0 * kDim[t]; i < i1 * kDim[t]; ++i) tp.isig[i] = 1.0 / b->sigmas[i];
      if (!tp.meas.empty())
        std::memcpy(tp.meas.data() + i0 * kMeasDim[t], b->measured + i0 * kMeasDim[t], (i1 - i0) * kMeasDim[t] * sizeof(double));
      for (int64_t i = i0; i < i1; ++i) tp.hk[i] = b->huber_k ? b->huber_k[i] : 0.0;
    });
  }

  if (hook) hook->types_ready(P);
  plan_mark("before point-pose edges", tmark);
  // ---- point-pose edges ----
  {
    // bucket (point, pose) incidences by point, then sort + unique each
    // point's (short) pose list: the (point, pose)-sorted unique edge list
    // (serial: shared counters on the workers measured slower on the GPU
    // box's host, whose cores do not share one cache)
    std::vector<int32_t>& cnt = sc.cnt;
    cnt.assign(P.n_pt + 1, 0);
    auto each = [&](auto&& fn) {
      for (int t = 0; t < kNTypes; ++t) {
        const TypePlan& tp = P.types[t];
        const int nk = kNKeys[t];
        for (int i = 0; i < tp.n; ++i)
          for (int sa = 0; sa < nk; ++sa)
            if (kSlotKind[t][sa] == 1)
              for (int sb = 0; sb < nk; ++sb)
                if (kSlotKind[t][sb] == 0) fn(tp.idx[i * nk + sa], tp.idx[i * nk + sb]);
      }
    };
    each([&](int32_t pt, int32_t) { cnt[pt + 1]++; });
    for (int i = 0; i < P.n_pt; ++i) cnt[i + 1] += cnt[i];
    auto& poses = sc.poses;
    poses.resize(cnt[P.n_pt]);
    {
      std::vector<int32_t> cur(cnt.begin(), cnt.end() - 1);
      each([&](int32_t pt, int32_t pose) { poses[cur[pt]++] = pose; });
    }
    // per point (in parallel): sort + unique its poses in place, then the
    // prefix of the unique counts places every point's edges
    P.pt_edge_start.assign(P.n_pt + 1, 0);
    parallel_for(P.n_pt, [&](int64_t p0, int64_t p1) {
      for (int64_t pt = p0; pt < p1; ++pt) {
        auto b = poses.begin() + cnt[pt], e = poses.begin() + cnt[pt + 1];
        std::sort(b, e);
        P.pt_edge_start[pt + 1] = static_cast<int32_t>(std::unique(b, e) - b);
      }
    });
    for (int pt = 0; pt < P.n_pt; ++pt) P.pt_edge_start[pt + 1] += P.pt_edge_start[pt];
    P.n_edge = P.pt_edge_start[P.n_pt];
    P.edge_pt.resize(P.n_edge);
    P.edge_pose.resize(P.n_edge);
    parallel_for(P.n_pt, [&](int64_t p0, int64_t p1) {
      for (int64_t pt = p0; pt < p1; ++pt) {
        const int32_t o = P.pt_edge_start[pt], k = P.pt_edge_start[pt + 1] - o;
        for (int32_t j = 0; j < k; ++j) {
          P.edge_pt[o + j] = static_cast<int32_t>(pt);
          P.edge_pose[o + j] = poses[cnt[pt] + j];
        }
      }
    });
  }
  auto find_edge = [&](int32_t pt, int32_t pose) -> int32_t {
    auto b = P.edge_pose.begin() + P.pt_edge_start[pt];
    auto e = P.edge_pose.begin() + P.pt_edge_start[pt + 1];
    auto it = std::lower_bound(b, e, pose);
    return static_cast<int32_t>(it - P.edge_pose.begin());
  };

  plan_mark("before arena layout", tmark);
  // ---- arena layout ----
  // every region starts at an even offset (16-byte aligned), so blocks at
  // even offsets inside it can be read with 16-byte loads
  auto align2 = [&arena] { arena = (arena + 1) & ~1ull; };
  P.off_D = arena; arena += 9ull * P.n_pt;
  align2();
  P.off_E = arena; arena += 9ull * P.n_pt;
  align2();
  P.off_gp = arena; arena += 3ull * P.n_pt;
  align2();
  P.off_W = arena; arena += 18ull * P.n_edge;

  plan_mark("before component neighbour poses and Y layout", tmark);
  // ---- component neighbour poses and Y layout ----
  P.comp_y_base.resize(P.n_comp);
  P.off_Y = arena;
  // chains of >= 2 points come first (longest first), the lone points last
  int32_t c_lone = 0;
  while (c_lone < P.n_comp && P.comp_start[c_lone + 1] - P.comp_start[c_lone] >= 2) ++c_lone;
  {
    // A chain's (neighbour pose, local point, edge) incidences sorted by
    // (pose, point): the distinct poses are its neighbour poses (ascending)
    // and each pose's run lists its edges in point order. Counted on the
    // workers, placed by a prefix over the chains, then filled on the
    // workers: the arrays equal the sequential layout.
    struct Inc {
      uint64_t key;   // pose << 32 | local point
      int32_t e;
    };
    auto incidences = [&](int c, std::vector<Inc>& inc) {
      inc.clear();
      for (int32_t i = P.comp_start[c]; i < P.comp_start[c + 1]; ++i)
        for (int32_t e = P.pt_edge_start[i]; e < P.pt_edge_start[i + 1]; ++e)
          inc.push_back(Inc{(static_cast<uint64_t>(P.edge_pose[e]) << 32) | static_cast<uint32_t>(i - P.comp_start[c]), e});
      std::sort(inc.begin(), inc.end(), [](const Inc& a, const Inc& b) { return a.key < b.key; });
    };
    std::vector<int32_t> chain_m(static_cast<size_t>(c_lone) + 1, 0);
    parallel_chunks(c_lone, 16, [&](int64_t c0, int64_t c1) {
      std::vector<Inc> inc;
      for (int64_t c = c0; c < c1; ++c) {
        incidences(static_cast<int>(c), inc);
        int32_t m = 0;
        for (size_t k = 0; k < inc.size(); ++k) m += k == 0 || (inc[k].key >> 32) != (inc[k - 1].key >> 32);
        chain_m[c + 1] = m;
      }
    });
    for (int c = 0; c < c_lone; ++c) {
      const int nc = P.comp_start[c + 1] - P.comp_start[c];
      P.comp_y_base[c] = static_cast<int64_t>(arena);
      arena += 18ull * nc * chain_m[c + 1];
      chain_m[c + 1] += chain_m[c];
    }
    P.comp_nb_start.assign(chain_m.begin(), chain_m.end());
    const int32_t n_nb = chain_m[c_lone];
    // a chain's points' edges are contiguous from its first point's first edge
    const int32_t n_nbe = c_lone > 0 ? P.pt_edge_start[P.comp_start[c_lone]] : 0;
    P.nb_pose.resize(n_nb);
    P.nb_comp.resize(n_nb);
    P.nbedge_start.resize(static_cast<size_t>(n_nb) + 1);
    P.nbedge_start[0] = 0;
    P.nbedge_pt.resize(n_nbe);
    P.nbedge_w.resize(n_nbe);
    parallel_chunks(c_lone, 16, [&](int64_t c0, int64_t c1) {
      std::vector<Inc> inc;
      for (int64_t c = c0; c < c1; ++c) {
        incidences(static_cast<int>(c), inc);
        int32_t b = chain_m[c] - 1;
        const int32_t q0 = P.pt_edge_start[P.comp_start[c]];
        for (size_t k = 0; k < inc.size(); ++k) {
          if (k == 0 || (inc[k].key >> 32) != (inc[k - 1].key >> 32)) {
            if (k > 0) P.nbedge_start[b + 1] = q0 + static_cast<int32_t>(k);
            ++b;
            P.nb_pose[b] = static_cast<int32_t>(inc[k].key >> 32);
            P.nb_comp[b] = static_cast<int32_t>(c);
          }
          P.nbedge_pt[q0 + k] = static_cast<int32_t>(inc[k].key & 0xffffffffu);
          P.nbedge_w[q0 + k] = static_cast<uint32_t>(P.off_W + 18ull * inc[k].e);
        }
        if (!inc.empty()) P.nbedge_start[b + 1] = q0 + static_cast<int32_t>(inc.size());
      }
    });
  }
  {
    // a lone point's neighbour poses are its (sorted, unique) edges, one edge
    // each; the lone points' edges are contiguous, so every position follows
    // from the edge index (filled in parallel)
    const int32_t e_l0 = c_lone < P.n_comp ? P.pt_edge_start[P.comp_start[c_lone]] : P.n_edge;
    const int64_t nl = P.n_edge - e_l0;
    const int64_t nb_base = static_cast<int64_t>(P.nb_pose.size()), ne_base = static_cast<int64_t>(P.nbedge_pt.size());
    P.nb_pose.resize(nb_base + nl);
    P.nb_comp.resize(nb_base + nl);
    P.nbedge_pt.resize(ne_base + nl);
    P.nbedge_w.resize(ne_base + nl);
    P.nbedge_start.resize(nb_base + nl + 1);
    P.comp_nb_start.resize(static_cast<size_t>(P.n_comp) + 1);
    const uint64_t y0 = arena;
    arena += 18ull * nl;
    parallel_for(P.n_comp - c_lone, [&](int64_t q0, int64_t q1) {
      for (int64_t q = q0; q < q1; ++q) {
        const int32_t c = c_lone + static_cast<int32_t>(q), i = P.comp_start[c];
        const int32_t e0 = P.pt_edge_start[i], e1 = P.pt_edge_start[i + 1];
        P.comp_y_base[c] = static_cast<int64_t>(y0 + 18ull * (e0 - e_l0));
        for (int32_t e = e0; e < e1; ++e) {
          const int64_t j = e - e_l0;
          P.nb_pose[nb_base + j] = P.edge_pose[e];
          P.nb_comp[nb_base + j] = c;
          P.nbedge_pt[ne_base + j] = 0;
          P.nbedge_w[ne_base + j] = static_cast<uint32_t>(P.off_W + 18ull * e);
          P.nbedge_start[nb_base + j + 1] = static_cast<int32_t>(ne_base + j + 1);
        }
        P.comp_nb_start[c + 1] = static_cast<int32_t>(nb_base + (e1 - e_l0));
      }
    });
  }
  P.off_v = arena; arena += 3ull * P.n_pt;
  align2();
  P.off_L = arena; arena += 9ull * P.n_pt;
  align2();
  P.off_M = arena; arena += 9ull * P.n_pt;
  P.arena_size = arena;
  if (arena >= (1ull << 32)) { err = "graph too large for 32-bit arena offsets"; return DYNOHIP_ESTRUCT; }

  plan_mark("before reduced system structure", tmark);
  // ---- reduced system structure ----
  // Pose-pair blocks (A >= B) of the reduced system: every diagonal (for the
  // damping), the pose pairs of every factor and the neighbour-pose pairs of
  // every point component, numbered in (B, A) order (band column order).
  // pair index: dense rows of width (max A - B) + 1 when that is small,
  // a hash map otherwise. The distinct pairs are the factor pose pairs and
  // the (a, b) neighbour pairs of every component (each neighbour pose has
  // at least one edge), so marking does not walk the edge lists.
  std::vector<int32_t> id_dense;
  std::unordered_map<uint64_t, int32_t> id_map;
  auto pkey = [](int32_t A, int32_t B) { return (static_cast<uint64_t>(B) << 32) | static_cast<uint32_t>(A); };
  int64_t span = 1;
  bool dense = true;
  auto each_distinct = [&](auto&& fn) {
    for (int t = 0; t < kNTypes; ++t) {
      const TypePlan& tp = P.types[t];
      const int nk = kNKeys[t];
      if (kNPoseSlots[t] < 2) continue;
      for (int i = 0; i < tp.n; ++i)
        for (int sa = 0; sa < nk; ++sa)
          if (kSlotKind[t][sa] == 0)
            for (int sb = 0; sb < nk; ++sb)
              if (kSlotKind[t][sb] == 0 && tp.idx[i * nk + sa] >= tp.idx[i * nk + sb])
                fn(tp.idx[i * nk + sa], tp.idx[i * nk + sb]);
    }
    for (int c = 0; c < P.n_comp; ++c) {
      const int32_t nb0 = P.comp_nb_start[c], m = P.comp_nb_start[c + 1] - nb0;
      for (int a = 0; a < m; ++a)
        for (int b = 0; b <= a; ++b) fn(P.nb_pose[nb0 + a], P.nb_pose[nb0 + b]);
    }
  };
  auto structure = [&] {
    int32_t W = 0;
    for (int t = 0; t < kNTypes; ++t) {
      const TypePlan& tp = P.types[t];
      const int nk = kNKeys[t];
      if (kNPoseSlots[t] < 2) continue;
      for (int i = 0; i < tp.n; ++i)
        for (int sa = 0; sa < nk; ++sa)
          for (int sb = 0; sb < nk; ++sb)
            if (kSlotKind[t][sa] == 0 && kSlotKind[t][sb] == 0)
              W = std::max(W, tp.idx[i * nk + sa] - tp.idx[i * nk + sb]);
    }
    for (int c = 0; c < P.n_comp; ++c) {  // nb poses are sorted per component
      const int32_t nb0 = P.comp_nb_start[c], nb1 = P.comp_nb_start[c + 1];
      if (nb1 > nb0) W = std::max(W, P.nb_pose[nb1 - 1] - P.nb_pose[nb0]);
    }
    span = static_cast<int64_t>(W) + 1;
    dense = static_cast<int64_t>(P.n_pose) * span <= (int64_t{1} << 26);
    if (dense) id_dense.assign(static_cast<size_t>(P.n_pose) * span, -1);
    auto mark = [&](int32_t A, int32_t B) {
      if (dense) id_dense[static_cast<size_t>(A) * span + (A - B)] = 0;
      else id_map.emplace(pkey(A, B), 0);
    };
    for (int32_t A = 0; A < P.n_pose; ++A) mark(A, A);
    each_distinct(mark);
    P.red_A.clear();
    P.red_B.clear();
    if (dense) {
      for (int32_t B = 0; B < P.n_pose; ++B)
        for (int32_t A = B; A < P.n_pose && A - B < span; ++A) {
          int32_t& id = id_dense[static_cast<size_t>(A) * span + (A - B)];
          if (id < 0) continue;
          id = static_cast<int32_t>(P.red_A.size());
          P.red_A.push_back(A);
          P.red_B.push_back(B);
        }
    } else {
      std::vector<uint64_t> ks;
      ks.reserve(id_map.size());
      for (const auto& kv : id_map) ks.push_back(kv.first);
      std::sort(ks.begin(), ks.end());  // (B, A) order
      for (uint64_t k : ks) {
        id_map[k] = static_cast<int32_t>(P.red_A.size());
        P.red_A.push_back(static_cast<int32_t>(k & 0xffffffffu));
        P.red_B.push_back(static_cast<int32_t>(k >> 32));
      }
    }
    // ---- band layout ----
    P.n_red = 6 * P.n_pose;
    P.NT = (P.n_red + kTile - 1) / kTile;
    std::vector<int32_t> rlow(P.NT);
    for (int j = 0; j < P.NT; ++j) rlow[j] = j;
    for (size_t t = 0; t < P.red_A.size(); ++t) {
      const int r1 = (6 * P.red_A[t] + 5) / kTile;
      const int c0 = (6 * P.red_B[t]) / kTile, c1 = (6 * P.red_B[t] + 5) / kTile;
      for (int j = c0; j <= c1; ++j) rlow[j] = std::max(rlow[j], r1);
    }
    for (int j = 1; j < P.NT; ++j) rlow[j] = std::max(rlow[j], rlow[j - 1]);
    P.band_D.resize(P.NT);
    P.max_D = 0;
    for (int j = 0; j < P.NT; ++j) {
      P.band_D[j] = rlow[j] - j;
      P.max_D = std::max(P.max_D, P.band_D[j]);
    }
  };
  // The pair structure, the band and then the tile schedule depend on the
  // factors' pose slots and the components' neighbour poses alone: they are
  // built on a thread of its own while this one builds the point-side lists
  // (the thread writes only its own Plan fields; the pair lists below wait
  // for the pair index, the target slots for the whole thread)
  std::promise<void> pairs_ready;
  std::future<void> pairs_done = pairs_ready.get_future();
  bool sched_ok = true;
  std::thread sched;
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } sched_join{sched};
  auto sched_body = [&] {
    PlanCap sched_cap(pcap);
    structure();
    pairs_ready.set_value();
    if (with_schedule) sched_ok = build_tile_schedule(P, true);
  };
  // a small graph's structure and schedule take less than starting and
  // joining a thread for them: run them here, first
  if (pcap == 1) sched_body();
  else sched = std::thread(sched_body);
  auto tid = [&](int32_t A, int32_t B) -> int32_t {
    return dense ? id_dense[static_cast<size_t>(A) * span + (A - B)] : id_map.at(pkey(A, B));
  };
  plan_mark("reduced system structure (started)", tmark);

  plan_mark("before point-side gathers", tmark);
  std::vector<uint8_t> lone_grouped(P.n_pt, 0);   // per point: in a lone-point group
  // ---- point-side gathers (CSR builds run on worker threads) ----
  // Point-slot references (type, factor, slot) in enumeration order
  // (type-major, then factor, then slot), stably sorted by point: a worker
  // owning a point range walks only its points' references, and every
  // target still lists its entries in factor order.
  bool chain_ok = true;
  if (!structure_only) {
    // (a serial counting sort: per-worker histograms scatter into shared
    // lines and measured slower on the GPU box's host)
    std::vector<int64_t>& rstart = sc.rstart;
    rstart.assign(static_cast<size_t>(P.n_pt) + 1, 0);
    for (int t = 0; t < kNTypes; ++t) {
      const TypePlan& tp = P.types[t];
      const int nk = kNKeys[t];
      for (int s = 0; s < nk; ++s)
        if (kSlotKind[t][s] == 1)
          for (int i = 0; i < tp.n; ++i) rstart[tp.idx[i * nk + s] + 1]++;
    }
    for (int32_t pt = 0; pt < P.n_pt; ++pt) rstart[pt + 1] += rstart[pt];
    auto& refs = sc.refs;
    refs.resize(rstart[P.n_pt]);
    {
      std::vector<int64_t> cur(rstart.begin(), rstart.end() - 1);
      for (int t = 0; t < kNTypes; ++t) {
        const TypePlan& tp = P.types[t];
        const int nk = kNKeys[t];
        for (int i = 0; i < tp.n; ++i)
          for (int s = 0; s < nk; ++s)
            if (kSlotKind[t][s] == 1)
              refs[cur[tp.idx[i * nk + s]]++] = (static_cast<uint64_t>(i) << 8) | (t << 4) | s;
      }
    }
    // a chain link (two point slots) must join consecutive points of one
    // component; its E entry goes to the lower point
    for (int t = 0; t < kNTypes; ++t) {
      const TypePlan& tp = P.types[t];
      const int nk = kNKeys[t];
      int ps[2], np = 0;
      for (int s = 0; s < nk; ++s)
        if (kSlotKind[t][s] == 1 && np < 2) ps[np++] = s;
      if (np != 2) continue;
      for (int i = 0; i < tp.n; ++i) {
        int32_t pa = tp.idx[i * nk + ps[0]], pb = tp.idx[i * nk + ps[1]];
        if (pa > pb) std::swap(pa, pb);
        if (pb != pa + 1 || comp_of[pa] != comp_of[pb]) chain_ok = false;
      }
    }
    if (!chain_ok) { err = "internal: chain link not adjacent"; return DYNOHIP_ESTRUCT; }
    plan_mark("point references by point", tmark);
    // the entries of points [p0, p1); `which` selects D (0), E (1), g_p (2) or W (3)
    auto emit_point = [&](int which, int32_t p0, int32_t p1, auto&& fn) {
      for (int32_t pt = p0; pt < p1; ++pt)
        for (int64_t q = rstart[pt]; q < rstart[pt + 1]; ++q) {
          const uint64_t r = refs[q];
          const int s = static_cast<int>(r & 15), t = static_cast<int>((r >> 4) & 15);
          const int i = static_cast<int>(r >> 8);
          const TypePlan& tp = P.types[t];
          const int nk = kNKeys[t], d = kDim[t];
          const uint32_t J = block_off(tp, t, i, s);
          if (which == 0) fn(pt, GEntry{J, J, d, 1});
          if (which == 2) fn(pt, GEntry{J, b_off(tp, t, i), d, 1});
          if (which == 3)
            for (int sb = 0; sb < nk; ++sb)
              if (kSlotKind[t][sb] == 0) fn(find_edge(pt, tp.idx[i * nk + sb]), GEntry{J, block_off(tp, t, i, sb), d, 1});
          if (which == 1) {
            int so = -1;
            for (int sb = 0; sb < nk; ++sb)
              if (kSlotKind[t][sb] == 1 && sb != s) so = sb;
            // E_pa = C_{pa+1, pa} = J_{pb}^T J_{pa}, once per link (from its lower point)
            if (so >= 0 && tp.idx[i * nk + so] == pt + 1) fn(pt, GEntry{block_off(tp, t, i, so), J, d, 1});
          }
        }
    };
    // ---- lone-point groups (plan.hpp LoneGroup) ----
    // Eligible: a lone point with 1..kLoneMaxNb neighbour poses and exactly
    // one PoseToPoint factor per neighbour (every static landmark of the
    // formulations). Grouped by the neighbour list (bucketed by its first
    // pose, then compared), in point order; a group is split into
    // near-equal subgroups of at most lone_cap(m) points.
    P.lgroup.clear();
    P.lone_pose.clear();
    P.lone_blk.clear();
    P.lone_max_m = 0;
    int32_t c_long = 0;
    while (c_long < P.n_comp && P.comp_start[c_long + 1] - P.comp_start[c_long] >= 2) ++c_long;
    const int32_t p_lone = c_long < P.n_comp ? P.comp_start[c_long] : P.n_pt;
    const int32_t e_l0 = p_lone < P.n_pt ? P.pt_edge_start[p_lone] : P.n_edge;
    const int32_t n_lone = P.n_pt - p_lone;
    std::vector<uint8_t> ok(static_cast<size_t>(n_lone), 0);
    std::vector<uint32_t>& prec = sc.prec;
    prec.assign(static_cast<size_t>(P.n_edge - e_l0), 0);
    const TypePlan& t0 = P.types[0];
    parallel_for(n_lone, [&](int64_t q0, int64_t q1) {
      for (int64_t q = q0; q < q1; ++q) {
        const int32_t pt = p_lone + static_cast<int32_t>(q);
        const int32_t e0 = P.pt_edge_start[pt], m = P.pt_edge_start[pt + 1] - e0;
        if (m < 1 || m > kLoneMaxNb || rstart[pt + 1] - rstart[pt] != m) continue;
        uint32_t seen = 0;
        bool good = true;
        for (int64_t k = rstart[pt]; k < rstart[pt + 1]; ++k) {
          const uint64_t r = refs[k];
          const int i = static_cast<int>(r >> 8);
          if (((r >> 4) & 15) != 0) { good = false; break; }
          const int a = find_edge(pt, t0.idx[2 * i]) - e0;
          if ((seen >> a) & 1u) { good = false; break; }
          seen |= 1u << a;
          prec[e0 - e_l0 + a] = block_off(t0, 0, i, 0);
        }
        ok[q] = good;
      }
    });
    plan_mark("lone-point eligibility", tmark);
    std::vector<int32_t> fstart(static_cast<size_t>(P.n_pose) + 1, 0), byfirst;
    for (int32_t q = 0; q < n_lone; ++q)
      if (ok[q]) fstart[P.edge_pose[P.pt_edge_start[p_lone + q]] + 1]++;
    for (int32_t x = 0; x < P.n_pose; ++x) fstart[x + 1] += fstart[x];
    byfirst.resize(fstart[P.n_pose]);
    {
      std::vector<int32_t> cur(fstart.begin(), fstart.end() - 1);
      for (int32_t q = 0; q < n_lone; ++q)
        if (ok[q]) byfirst[cur[P.edge_pose[P.pt_edge_start[p_lone + q]]]++] = p_lone + q;
    }
    auto same_list = [&](int32_t u, int32_t v) {
      const int32_t eu = P.pt_edge_start[u], ev = P.pt_edge_start[v], m = P.pt_edge_start[u + 1] - eu;
      if (P.pt_edge_start[v + 1] - ev != m) return false;
      for (int32_t a = 0; a < m; ++a)
        if (P.edge_pose[eu + a] != P.edge_pose[ev + a]) return false;
      return true;
    };
    align2();
    P.off_I6 = arena;
    arena += 36;
    // per first-pose bucket: class representatives, each point's class, and
    // the members of one class at a time (flat scratch, no per-bucket allocation)
    std::vector<int32_t> rep, cls_of, mem;
    P.lone_blk.reserve(static_cast<size_t>(kLoneBlk) * (byfirst.size() / kLoneSub + 2 * static_cast<size_t>(P.n_pose) + 1));
    int64_t n_grouped = 0;
    for (int32_t x = 0; x < P.n_pose; ++x) {
      const int32_t k0b = fstart[x], k1b = fstart[x + 1];
      if (k0b == k1b) continue;
      rep.clear();
      cls_of.resize(k1b - k0b);
      for (int32_t k = k0b; k < k1b; ++k) {
        const int32_t pt = byfirst[k];
        size_t ci = 0;
        while (ci < rep.size() && !same_list(rep[ci], pt)) ++ci;
        if (ci == rep.size()) rep.push_back(pt);
        cls_of[k - k0b] = static_cast<int32_t>(ci);
      }
      for (size_t ci = 0; ci < rep.size(); ++ci) {
        mem.clear();
        for (int32_t k = k0b; k < k1b; ++k)
          if (cls_of[k - k0b] == static_cast<int32_t>(ci)) mem.push_back(byfirst[k]);
        const int32_t e0 = P.pt_edge_start[mem[0]], m = P.pt_edge_start[mem[0] + 1] - e0;
        const int32_t cap = lone_cap(m);
        const int32_t n = static_cast<int32_t>(mem.size()), nsub = (n + cap - 1) / cap;
        for (int32_t u = 0; u < nsub; ++u) {
          const int32_t k0 = static_cast<int32_t>(int64_t{n} * u / nsub), k1 = static_cast<int32_t>(int64_t{n} * (u + 1) / nsub);
          LoneGroup G;
          G.m = m;
          G.npt = k1 - k0;
          G.pose_beg = static_cast<int32_t>(P.lone_pose.size());
          G.out = static_cast<uint32_t>(arena);
          // the per-try partial blocks and gradients (k_lone_schur), then the
          // H area of the fused linearisation (k_lone_lin: 6x6 J_a^T J_a and
          // J_a^T b per neighbour)
          arena += 36ull * (m * (m + 1) / 2) + 6ull * m + 42ull * m;
          P.lone_max_m = std::max(P.lone_max_m, m);
          for (int32_t a = 0; a < m; ++a) P.lone_pose.push_back(P.edge_pose[e0 + a]);
          const size_t bo = P.lone_blk.size();
          P.lone_blk.resize(bo + kLoneBlk);
          int32_t* blk = P.lone_blk.data() + bo;
          std::fill(blk, blk + kLoneBlk, 0);
          blk[0] = m;
          blk[1] = G.npt;
          blk[2] = static_cast<int32_t>(G.out);
          for (int32_t a = 0; a < m; ++a) blk[kLoneHdrPose + a] = P.edge_pose[e0 + a];
          for (int32_t k = k0; k < k1; ++k) {
            const int32_t pt = mem[k], u = k - k0;
            blk[kLoneHdrPt + u] = pt;
            blk[kLoneHdrE0 + u] = P.pt_edge_start[pt];
            lone_grouped[pt] = 1;
            const int32_t ep = P.pt_edge_start[pt] - e_l0;
            for (int32_t a = 0; a < m; ++a) blk[kLoneHdrRec + m * u + a] = static_cast<int32_t>(prec[ep + a]);
          }
          P.lgroup.push_back(G);
        }
        n_grouped += n;
      }
    }
    P.lone_all_grouped = n_grouped == n_lone;
    P.arena_size = arena;
    if (arena >= (1ull << 32)) { err = "graph too large for 32-bit arena offsets"; return DYNOHIP_ESTRUCT; }
    // with every lone point grouped, their D, g_p and W come from the
    // group blocks (k_gather_point's lone blocks): the CSR gathers stop at
    // the first lone point / edge (E stays whole: lone points have none)
    plan_mark("lone-point groups", tmark);
    const int32_t pt_end = P.lone_all_grouped ? p_lone : P.n_pt;
    const int32_t edge_end = P.lone_all_grouped ? e_l0 : P.n_edge;
    for (int which = 0; which < 4; ++which) {
      GatherList& out = which == 0 ? P.gD : which == 1 ? P.gE : which == 2 ? P.gGp : P.gW;
      const int64_t nt = which == 3 ? edge_end : which == 1 ? P.n_pt : pt_end;
      const std::vector<int64_t> cut = even_cuts(nt);
      csr_target_ranges(nt, cut,
                        [&](int r, auto&& fn) {
                          if (cut[r + 1] <= cut[r]) return;
                          if (which != 3) {
                            emit_point(which, static_cast<int32_t>(cut[r]), static_cast<int32_t>(cut[r + 1]), fn);
                          } else {
                            emit_point(which, P.edge_pt[cut[r]], P.edge_pt[cut[r + 1] - 1] + 1, fn);
                          }
                        },
                        out);
    }

  }


  pairs_done.wait();
  plan_mark("before reduced system targets (pair index wait)", tmark);
  // ---- reduced system targets ----
  // Pose-pair blocks (A >= B) of the reduced system: every diagonal (for the
  // damping), the pose pairs of every factor and the neighbour-pose pairs of
  // every point component. Targets are numbered in (B, A) order (band column
  // order); each target's entries keep the enumeration order below.
  {
    // the pair enumeration: the factors' pose pairs, then every component's
    // neighbour-pose pairs, components in order
    // the PoseToPoint factors outside the lone groups, in factor order (the
    // enumerations below run once per worker and pass: they skip the grouped
    // ones without visiting them)
    std::vector<int32_t>& keep0 = P.lin_list0;
    keep0.clear();
    {
      // (an ordered filter on the workers: count per chunk, then fill)
      const int64_t n0 = P.types[0].n;
      const int nw = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(PlanPool::get().workers(), n0 / 16384 + 1)));
      std::vector<int64_t> kc(static_cast<size_t>(nw) + 1, 0);
      auto keep = [&](int64_t i) { return !lone_grouped[P.types[0].idx[2 * i + 1]]; };
      PlanPool::get().run(nw, [&](int w) {
        int64_t c = 0;
        for (int64_t i = n0 * w / nw; i < n0 * (w + 1) / nw; ++i) c += keep(i);
        kc[w + 1] = c;
      });
      for (int w = 0; w < nw; ++w) kc[w + 1] += kc[w];
      keep0.resize(kc[nw]);
      PlanPool::get().run(nw, [&](int w) {
        int64_t o = kc[w];
        for (int64_t i = n0 * w / nw; i < n0 * (w + 1) / nw; ++i)
          if (keep(i)) keep0[o++] = static_cast<int32_t>(i);
      });
    }
    auto comp_grouped = [&](int c) {
      return P.comp_start[c + 1] - P.comp_start[c] == 1 && lone_grouped[P.comp_start[c]];
    };
    // pose pairs (A >= B) of factor i of type t
    auto factor_pairs = [&](int t, int i, auto&& pair_fn) {  // pair_fn(A, B, entry)
      const TypePlan& tp = P.types[t];
      const int nk = kNKeys[t], d = kDim[t];
      for (int sa = 0; sa < nk; ++sa) {
        if (kSlotKind[t][sa] != 0) continue;
        const int32_t A = tp.idx[i * nk + sa];
        for (int sb = 0; sb < nk; ++sb) {
          if (kSlotKind[t][sb] != 0) continue;
          const int32_t B = tp.idx[i * nk + sb];
          if (A < B) continue;
          pair_fn(A, B, GEntry{block_off(tp, t, i, sa), block_off(tp, t, i, sb), d, 1});
        }
      }
    };
    // the neighbour-pose pairs of component c
    auto emit_comp_pairs = [&](int c, auto&& pair_fn) {
      const int32_t nb0 = P.comp_nb_start[c], m = P.comp_nb_start[c + 1] - nb0;
      for (int a = 0; a < m; ++a) {
        const int32_t A = P.nb_pose[nb0 + a];
        for (int b = 0; b <= a; ++b) {
          const int32_t B = P.nb_pose[nb0 + b];
          for (int32_t q = P.nbedge_start[nb0 + a]; q < P.nbedge_start[nb0 + a + 1]; ++q) {
            const int i = P.nbedge_pt[q];
            const uint32_t y = static_cast<uint32_t>(P.comp_y_base[c] + 18ll * (static_cast<int64_t>(i) * m + b));
            pair_fn(A, B, GEntry{P.nbedge_w[q], y, 3, -1});
          }
        }
      }
    };
    // The sources of both reduced-system lists in enumeration order: the
    // factors (type-major, each type in factor order; the PoseToPoint factors
    // of grouped lone points are left out, their blocks come through the
    // groups), then the components (grouped lone points and components
    // without neighbour poses emit nothing), then the lone-point groups.
    int64_t ffirst[kNTypes + 1];
    ffirst[0] = 0;
    for (int t = 0; t < kNTypes; ++t)
      ffirst[t + 1] = ffirst[t] + (t == 0 ? static_cast<int64_t>(keep0.size()) : P.types[t].n);
    const int64_t nF = ffirst[kNTypes], nC = P.n_comp, nG = static_cast<int64_t>(P.lgroup.size());
    const int64_t nsrc = nF + nC + nG;
    auto visit = [&](int64_t s0, int64_t s1, auto&& on_factor, auto&& on_comp, auto&& on_group) {
      for (int t = 0; t < kNTypes; ++t)
        for (int64_t s = std::max(s0, ffirst[t]); s < std::min(s1, ffirst[t + 1]); ++s)
          on_factor(t, t == 0 ? keep0[s] : static_cast<int>(s - ffirst[t]));
      for (int64_t s = std::max(s0, nF); s < std::min(s1, nF + nC); ++s) {
        const int c = static_cast<int>(s - nF);
        if (P.comp_nb_start[c + 1] == P.comp_nb_start[c] || comp_grouped(c)) continue;
        on_comp(c);
      }
      for (int64_t s = std::max(s0, nF + nC); s < s1; ++s) on_group(P.lgroup[s - nF - nC]);
    };
    if (!structure_only) {
      std::thread grad;
      auto grad_body = [&] {
        PlanCap grad_cap(pcap);
        // gradient gathers per pose: J_A^T b per factor, -W_A v per component,
        // the groups' partial gradients
        // (on a thread of its own, one range: it runs beside the pair lists)
        const std::vector<int64_t> gcut{0, P.n_pose};
        csr_target_ranges(P.n_pose, gcut,
                          [&](int r, auto&& fn) {
                            const int64_t p0 = gcut[r], p1 = gcut[r + 1];
                            visit(0, nsrc,
                                  [&](int t, int i) {
                                    const TypePlan& tp = P.types[t];
                                    const int nk = kNKeys[t], d = kDim[t];
                                    for (int sa = 0; sa < nk; ++sa)
                                      if (kSlotKind[t][sa] == 0)
                                        fn(tp.idx[i * nk + sa], GEntry{block_off(tp, t, i, sa), b_off(tp, t, i), d, 1});
                                  },
                                  [&](int c) {
                                    const int32_t nb0 = P.comp_nb_start[c], m = P.comp_nb_start[c + 1] - nb0;
                                    if (P.nb_pose[nb0 + m - 1] < p0 || P.nb_pose[nb0] >= p1) return;
                                    for (int a = 0; a < m; ++a)
                                      for (int32_t q = P.nbedge_start[nb0 + a]; q < P.nbedge_start[nb0 + a + 1]; ++q)
                                        fn(P.nb_pose[nb0 + a],
                                           GEntry{P.nbedge_w[q],
                                                  static_cast<uint32_t>(P.off_v + 3ull * (P.comp_start[c] + P.nbedge_pt[q])), 3, -1});
                                  },
                                  [&](const LoneGroup& G) {
                                    const int32_t* ps = P.lone_pose.data() + G.pose_beg;
                                    if (ps[G.m - 1] < p0 || ps[0] >= p1) return;
                                    const uint32_t g0 = G.out + 36u * (G.m * (G.m + 1) / 2);
                                    for (int a = 0; a < G.m; ++a)
                                      fn(ps[a], GEntry{static_cast<uint32_t>(P.off_I6), g0 + 6u * a, 6, kAddBlock});
                                  });
                          },
                          P.gGred);
      };
      if (pcap == 1) grad_body();
      else grad = std::thread(grad_body);
      struct JoinGrad {
        std::thread& t;
        ~JoinGrad() {
          if (t.joinable()) t.join();
        }
      } grad_join{grad};
      // J_A^T J_B per factor pair, -W_A Y_B per component pair, the groups'
      // partial blocks
      // target ranges: worker r owns the targets of a B range and enumerates
      // every source, skipping components and groups outside its range;
      // each worker writes one contiguous part of the list
      const std::vector<int64_t> rcut = even_cuts(static_cast<int64_t>(P.red_A.size()));
      csr_target_ranges(P.red_A.size(), rcut,
                        [&](int r, auto&& fn) {
                          if (rcut[r + 1] <= rcut[r]) return;
                          const int32_t blo = P.red_B[rcut[r]], bhi = P.red_B[rcut[r + 1] - 1];
                          auto pf = [&](int32_t A, int32_t B, const GEntry& e) {
                            if (B >= blo && B <= bhi) fn(tid(A, B), e);
                          };
                          visit(0, nsrc, [&](int t, int i) { factor_pairs(t, i, pf); },
                                [&](int c) {
                                  const int32_t nb0 = P.comp_nb_start[c], nb1 = P.comp_nb_start[c + 1];
                                  if (P.nb_pose[nb1 - 1] < blo || P.nb_pose[nb0] > bhi) return;
                                  emit_comp_pairs(c, pf);
                                },
                                [&](const LoneGroup& G) {
                                  const int32_t* ps = P.lone_pose.data() + G.pose_beg;
                                  if (ps[G.m - 1] < blo || ps[0] > bhi) return;
                                  for (int a = 0; a < G.m; ++a)
                                    for (int b = 0; b <= a; ++b)
                                      pf(ps[a], ps[b], GEntry{static_cast<uint32_t>(P.off_I6),
                                                              G.out + 36u * (a * (a + 1) / 2 + b), 6, kAddBlock});
                                });
                        },
                        P.gRed);
      if (grad.joinable()) grad.join();
    }
  }
  plan_mark("reduced system targets", tmark);

  if (sched.joinable()) sched.join();
  if (with_schedule && !sched_ok) {
    err = "graph too short in time for " + std::to_string(nranks) + " partitions";
    return DYNOHIP_ESTRUCT;
  }
  plan_mark("tile schedule (join)", tmark);
  if (with_schedule && !structure_only) compute_red_slots(P);
  plan_mark("reduced target slots", tmark);
  return DYNOHIP_OK;
}

}  // namespace dynohip
