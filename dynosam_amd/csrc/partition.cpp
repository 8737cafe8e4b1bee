// partition.cpp — the full-batch graph split over ranks for the partitioned
// Schur solve (BASELINE configs[4]: "landmark-block
// partitioned Schur with RCCL reduce of reduced system").
//
// The reference solves the whole graph in one GTSAM process
// (RGBDBackendModule.cc:207-231). Here the nested dissection of the reduced
// pose system (tiles.cpp) is forced to split its top log2(nranks) levels, so
// rank r owns one time-contiguous subtree of tiles (its interior) and each
// separator of those splits is a node owned by the group of ranks whose
// subtrees it splits. A factor that touches an interior tile of r, and every
// factor of a landmark chain that does, is linearised and Schur-eliminated on
// r only; the separators' dissection guarantees no factor or chain touches
// two interiors. Factors touching only one separator's tiles go to the
// leader (lowest rank) of its group. Every rank holds all poses (the reduced
// system keeps global numbering) and only its own landmarks.
//
// Per LM solve each rank eliminates its landmarks and its interior columns
// locally; then, level by level from the deepest separators up, the ranks
// sum the separator systems of that depth (one all-reduce per depth) and each
// group factors its own separator (solver.cpp), the leader passing the
// separator's contributions on to the separators above.
#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "plan.hpp"
#include "plan_pool.hpp"

namespace dynohip {

dynohip_graph_view GraphStore::view() const {
  dynohip_graph_view g;
  std::memset(&g, 0, sizeof(g));
  dynohip_factor_block* b[kNTypes] = {&g.pose_to_point, &g.landmark_motion_ternary, &g.between,
                                      &g.prior, &g.landmark_motion_pose, &g.landmark_pose_smoothing};
  for (int t = 0; t < kNTypes; ++t) {
    b[t]->n = n[t];
    b[t]->keys = keys[t].empty() ? nullptr : keys[t].data();
    b[t]->measured = meas[t].empty() ? nullptr : meas[t].data();
    b[t]->sigmas = sig[t].empty() ? nullptr : sig[t].data();
    b[t]->huber_k = hub[t].empty() ? nullptr : hub[t].data();
  }
  return g;
}

namespace {

// owner merge over the tiles a factor or chain touches: a rank (its
// interior) wins over a separator node (one of the rank's ancestors: a
// separator is adjacent only to the subtrees it splits); of two separator
// nodes on one root path the deeper one wins (a left subtree's reach is
// clipped at its end, so a depth-2 separator's tiles can neighbour the top
// separator's: the deeper node's leader is a member of every ancestor's
// group, and the ancestor's slots are exchanged at their own, later depth);
// two ranks, or two separator nodes on different paths, conflict
constexpr int32_t kOwnNone = INT32_MIN, kOwnConflict = INT32_MIN + 1;
int32_t merge_owner(int32_t a, int32_t b, const std::vector<SepNode>& nodes) {
  if (a == kOwnNone) return b;
  if (b == kOwnNone) return a;
  if (a == kOwnConflict || b == kOwnConflict) return kOwnConflict;
  if (a == b) return a;
  if (a >= 0 && b >= 0) return kOwnConflict;
  if (a >= 0) return a;
  if (b >= 0) return b;
  const SepNode& na = nodes[sep_node(a)];
  const SepNode& nb = nodes[sep_node(b)];
  auto within = [](const SepNode& in, const SepNode& out) {
    return in.r0 >= out.r0 && in.r0 + in.nr <= out.r0 + out.nr;
  };
  if (within(na, nb)) return a;   // a is the deeper node of the path
  if (within(nb, na)) return b;
  return kOwnConflict;
}

}  // namespace

int build_partitioned_plan(const dynohip_graph_view& g, const uint64_t* keys, const uint8_t* kind, size_t n,
                           int nranks, int rank, Plan& L, Partition& part, GraphStore& lg, std::string& err) {
  if (nranks < 2 || (nranks & (nranks - 1)) != 0 || rank < 0 || rank >= nranks) {
    err = "partitioned solve needs a power-of-two rank count >= 2 and 0 <= rank < nranks";
    return DYNOHIP_EINVAL;
  }
  // the global graph's structure (point chains, reduced system, the
  // partitioned tile schedule) without its gather lists: this rank's own
  // plan below builds those for its share only
  static const bool timing = std::getenv("DYNOHIP_PLAN_TIMING") != nullptr;
  auto t0 = std::chrono::steady_clock::now();
  auto mark = [&](const char* what) {
    const auto t = std::chrono::steady_clock::now();
    if (timing) std::fprintf(stderr, "[part] %-40s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - t0).count());
    t0 = t;
  };
  // The global structure first; its tile schedule then runs on a thread of
  // its own while this rank's share and local plan are built (the owners
  // they need follow from the pose-pair structure alone)
  Plan G;
  int rc = build_plan(g, keys, kind, n, G, err, nranks, rank, false, true);
  if (rc) return rc;
  std::vector<int32_t> towner;
  std::vector<SepNode> nodes;
  if (!partition_tile_owners(G, nranks, towner, nodes)) {
    err = "graph too short in time for " + std::to_string(nranks) + " partitions";
    return DYNOHIP_ESTRUCT;
  }
  bool sched_ok = true;
  std::thread sched([&G, &sched_ok] { sched_ok = build_tile_schedule(G, true); });
  struct Joiner {
    std::thread& t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } sched_join{sched};
  mark("global structure, owners");
  part = Partition();
  part.nranks = nranks;
  part.rank = rank;
  auto pose_owner = [&](int32_t p) {
    int32_t o = kOwnNone;
    for (int t = (6 * p) / kTile; t <= (6 * p + 5) / kTile; ++t) o = merge_owner(o, towner[t], nodes);
    return o;
  };
  // a separator node's factors and chains go to its group's leader
  // (a conflict maps to rank 0 here; the caller reports it as an error)
  auto to_rank = [&](int32_t o) {
    return o >= 0 ? o : (o == kOwnNone || o == kOwnConflict) ? 0 : nodes[sep_node(o)].r0;
  };
  std::vector<int32_t> comp_of(G.n_pt);
  parallel_for(G.n_comp, [&](int64_t c0, int64_t c1) {
    for (int64_t c = c0; c < c1; ++c)
      for (int32_t i = G.comp_start[c]; i < G.comp_start[c + 1]; ++i) comp_of[i] = static_cast<int32_t>(c);
  });
  // pass 1: every factor's pose owner (on the workers), then landmark chains
  // take the union of their factors' pose owners
  std::vector<int32_t> comp_own(G.n_comp, kOwnNone);
  std::vector<int32_t> fown[kNTypes];
  for (int t = 0; t < kNTypes; ++t) {
    const TypePlan& tp = G.types[t];
    const int nk = kNKeys[t];
    fown[t].resize(tp.n);
    parallel_for(tp.n, [&](int64_t i0, int64_t i1) {
      for (int64_t i = i0; i < i1; ++i) {
        int32_t o = kOwnNone;
        for (int sl = 0; sl < nk; ++sl)
          if (kSlotKind[t][sl] == 0) o = merge_owner(o, pose_owner(tp.idx[i * nk + sl]), nodes);
        fown[t][i] = o;
      }
    });
    for (int i = 0; i < tp.n; ++i)
      for (int sl = 0; sl < nk; ++sl)
        if (kSlotKind[t][sl] == 1) {
          const int c = comp_of[tp.idx[i * nk + sl]];
          comp_own[c] = merge_owner(comp_own[c], fown[t][i], nodes);
        }
  }
  for (int c = 0; c < G.n_comp; ++c) {
    if (comp_own[c] == kOwnConflict) {
      err = "internal: a landmark chain spans two partitions";
      return DYNOHIP_ESTRUCT;
    }
    comp_own[c] = to_rank(comp_own[c]);   // separator-only chains: the node's leader
  }
  // pass 2: factor owners, the local graph in the global factor order (an
  // ordered filter on the workers: owners and counts per chunk, then each
  // chunk's factors copied to their place)
  const dynohip_factor_block* gb[kNTypes] = {&g.pose_to_point, &g.landmark_motion_ternary, &g.between,
                                             &g.prior, &g.landmark_motion_pose, &g.landmark_pose_smoothing};
  lg = GraphStore();
  for (int t = 0; t < kNTypes; ++t) {
    const TypePlan& tp = G.types[t];
    const int nk = kNKeys[t], md = kMeasDim[t], dd = kDim[t];
    const int64_t nt = tp.n;
    const int nw = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(PlanPool::get().workers(), nt / 8192 + 1)));
    std::vector<int64_t> cnt(static_cast<size_t>(nw) + 1, 0);
    std::vector<uint8_t> bad(static_cast<size_t>(nw), 0);
    PlanPool::get().run(nw, [&](int w) {
      int64_t c = 0;
      for (int64_t i = nt * w / nw; i < nt * (w + 1) / nw; ++i) {
        int32_t o = fown[t][i];
        for (int sl = 0; sl < nk; ++sl)
          if (kSlotKind[t][sl] == 1) o = merge_owner(o, comp_own[comp_of[tp.idx[i * nk + sl]]], nodes);
        if (o == kOwnConflict) bad[w] = 1;
        o = to_rank(o);
        fown[t][i] = o;
        c += o == rank;
      }
      cnt[w + 1] = c;
    });
    for (int w = 0; w < nw; ++w)
      if (bad[w]) {
        err = "internal: a factor spans two partitions";
        return DYNOHIP_ESTRUCT;
      }
    for (int w = 0; w < nw; ++w) cnt[w + 1] += cnt[w];
    const int64_t nl = cnt[nw];
    part.factors_total += nt;
    part.factors_local += nl;
    lg.n[t] = nl;
    lg.keys[t].resize(nl * nk);
    lg.meas[t].resize(nl * md);
    lg.sig[t].resize(nl * dd);
    lg.hub[t].resize(nl);
    PlanPool::get().run(nw, [&](int w) {
      int64_t o = cnt[w];
      for (int64_t i = nt * w / nw; i < nt * (w + 1) / nw; ++i) {
        if (fown[t][i] != rank) continue;
        std::memcpy(lg.keys[t].data() + o * nk, gb[t]->keys + i * nk, nk * sizeof(uint64_t));
        if (md) std::memcpy(lg.meas[t].data() + o * md, gb[t]->measured + i * md, md * sizeof(double));
        std::memcpy(lg.sig[t].data() + o * dd, gb[t]->sigmas + i * dd, dd * sizeof(double));
        lg.hub[t][o] = gb[t]->huber_k ? gb[t]->huber_k[i] : 0.0;
        ++o;
      }
    });
  }
  // values: every pose, this rank's landmarks. A value's owner is the rank
  // that solves it and hands it back (a separator pose: its node's leader)
  part.value_owner.assign(n, -1);
  part.local_of.assign(n, -1);
  for (size_t v = 0; v < n; ++v) {
    const int32_t li = G.user_idx[v];
    const int32_t o = kind[v] == DYNOHIP_POSE3 ? to_rank(pose_owner(li)) : comp_own[comp_of[li]];
    part.value_owner[v] = o;
    if (kind[v] == DYNOHIP_POSE3 || o == rank) {
      part.local_of[v] = static_cast<int32_t>(part.keys.size());
      part.keys.push_back(keys[v]);
      part.kind.push_back(kind[v]);
      part.global_of.push_back(static_cast<int32_t>(v));
    }
  }
  mark("owners, local graph and values");
  const dynohip_graph_view lv = lg.view();
  rc = build_plan(lv, part.keys.data(), part.kind.data(), part.keys.size(), L, err, nranks, rank, false);
  if (rc) return rc;
  mark("local plan");
  sched.join();
  if (!sched_ok) {
    err = "graph too short in time for " + std::to_string(nranks) + " partitions";
    return DYNOHIP_ESTRUCT;
  }
  if (G.tile_owner != towner) {
    err = "internal: tile owners differ from the schedule's";
    return DYNOHIP_ESTRUCT;
  }
  mark("global schedule (join)");
  if (L.n_pose != G.n_pose || L.NT != G.NT || L.pose_key != G.pose_key) {
    err = "internal: local pose numbering differs from the global one";
    return DYNOHIP_ESTRUCT;
  }
  // the global partitioned schedule
  L.nd_leaf = G.nd_leaf;
  L.tile_pos = std::move(G.tile_pos);
  L.n_slots = G.n_slots;
  L.row_start = std::move(G.row_start);
  L.row_col = std::move(G.row_col);
  L.row_slot = std::move(G.row_slot);
  L.ftask = std::move(G.ftask);
  L.pairs = std::move(G.pairs);
  L.flevel = std::move(G.flevel);
  L.fpanels = std::move(G.fpanels);
  L.fdep_start = std::move(G.fdep_start);
  L.fdep = std::move(G.fdep);
  L.fqueue = std::move(G.fqueue);
  L.btask = std::move(G.btask);
  L.blevel = std::move(G.blevel);
  L.bent = std::move(G.bent);
  L.back_part_tiles = G.back_part_tiles;
  L.bpart = std::move(G.bpart);
  L.bplevel = std::move(G.bplevel);
  L.n_partials = G.n_partials;
  L.tile_flops = G.tile_flops;
  L.tile_owner = std::move(G.tile_owner);
  L.sep_nodes = std::move(G.sep_nodes);
  L.phases = std::move(G.phases);
  L.rhs0_tile = std::move(G.rhs0_tile);
  L.rhs0_start = std::move(G.rhs0_start);
  L.rhs0_slot = std::move(G.rhs0_slot);
  L.band_D = std::move(G.band_D);
  L.max_D = G.max_D;
  compute_red_slots(L);
  // damping: interior rows by their owner, separator rows by the node's
  // leader (the ranks' diagonals are summed in the exchange)
  mark("schedule into the local plan");
  part.damp_row.assign(static_cast<size_t>(L.n_red), 0);
  for (int q = 0; q < L.n_red; ++q) part.damp_row[q] = to_rank(L.tile_owner[q / kTile]) == rank ? 1 : 0;
  return DYNOHIP_OK;
}

}  // namespace dynohip

// Host-only introspection of the partitioned plan (tests/test_partition.py
// replays it in numpy): one named int32 array of rank `rank`'s plan.
extern "C" int dynohip_plan_export(const dynohip_graph_view* g, const uint64_t* keys, const uint8_t* kind, size_t n,
                                   int nranks, int rank, const char* name, int32_t* out, size_t cap,
                                   size_t* n_out) {
  using namespace dynohip;
  if (!g || !name || !n_out || (n && (!keys || !kind))) return DYNOHIP_EINVAL;
  Plan P;
  Partition part;
  GraphStore lg;
  std::string err;
  std::string nm(name);
  // "<name>@recycled": the plan built twice into one Plan object (the second
  // build reuses the first's arrays, plan_recycle), then exported
  const bool twice = nm.size() > 9 && nm.compare(nm.size() - 9, 9, "@recycled") == 0;
  if (twice) nm.resize(nm.size() - 9);
  for (int b = 0; b < (twice ? 2 : 1); ++b) {
    const int rc = nranks > 1 ? build_partitioned_plan(*g, keys, kind, n, nranks, rank, P, part, lg, err)
                              : build_plan(*g, keys, kind, n, P, err);
    if (rc) return rc;
  }
  std::vector<int32_t> tmp;
  const int32_t* src = nullptr;
  size_t cnt = 0;
  auto vec = [&](const std::vector<int32_t>& v) {
    src = v.data();
    cnt = v.size();
  };
  auto raw = [&](const void* p, size_t bytes) {
    src = static_cast<const int32_t*>(p);
    cnt = bytes / 4;
  };
  if (nm == "info") {
    tmp = {P.n_pose, P.NT, P.n_slots, P.nd_leaf, P.n_pt, static_cast<int32_t>(part.factors_local),
           static_cast<int32_t>(part.factors_total)};
    vec(tmp);
  } else if (nm == "tile_pos") vec(P.tile_pos);
  else if (nm == "tile_owner") vec(P.tile_owner);
  else if (nm == "pose_key") raw(P.pose_key.data(), P.pose_key.size() * sizeof(uint64_t));   // reduced pose order
  else if (nm == "row_start") vec(P.row_start);
  else if (nm == "row_col") vec(P.row_col);
  else if (nm == "row_slot") vec(P.row_slot);
  else if (nm == "pairs") vec(P.pairs);
  else if (nm == "ftask") raw(P.ftask.data(), P.ftask.size() * sizeof(TileTask));
  else if (nm == "flevel") vec(P.flevel);
  else if (nm == "fdep_start") vec(P.fdep_start);
  else if (nm == "fdep") vec(P.fdep);
  else if (nm == "fqueue") vec(P.fqueue);
  else if (nm == "sep_nodes") raw(P.sep_nodes.data(), P.sep_nodes.size() * sizeof(SepNode));
  // phase p of the separator phases (deepest first): "phase<p>_<field>", and
  // "phases": per phase (node, leader)
  else if (nm == "phases") {
    for (const PartPhase& F : P.phases) {
      tmp.push_back(F.node);
      tmp.push_back(F.leader);
    }
    vec(tmp);
  } else if (nm.size() > 7 && nm.compare(0, 5, "phase") == 0 && nm.find('_') != std::string::npos) {
    const size_t us = nm.find('_');
    const int ph = std::atoi(nm.substr(5, us - 5).c_str());
    if (ph < 0 || ph >= static_cast<int>(P.phases.size())) return DYNOHIP_EINVAL;
    const PartPhase& F = P.phases[ph];
    const std::string f = nm.substr(us + 1);
    if (f == "ftask") raw(F.ftask.data(), F.ftask.size() * sizeof(TileTask));
    else if (f == "flevel") vec(F.flevel);
    else if (f == "fdep_start") vec(F.fdep_start);
    else if (f == "fdep") vec(F.fdep);
    else if (f == "fqueue") vec(F.fqueue);
    else if (f == "xslot") vec(F.xslot);
    else if (f == "xtile") vec(F.xtile);
    else if (f == "rhs_tile") vec(F.rhs_tile);
    else if (f == "rhs_start") vec(F.rhs_start);
    else if (f == "rhs_slot") vec(F.rhs_slot);
    else return DYNOHIP_EINVAL;
  }
  else if (nm == "rhs0_tile") vec(P.rhs0_tile);
  else if (nm == "rhs0_start") vec(P.rhs0_start);
  else if (nm == "rhs0_slot") vec(P.rhs0_slot);
  else if (nm == "bpart") raw(P.bpart.data(), P.bpart.size() * sizeof(BackPart));
  else if (nm == "bplevel") vec(P.bplevel);
  else if (nm == "bent") vec(P.bent);
  else if (nm == "red_a") vec(P.red_A);
  else if (nm == "red_order") vec(P.red_order);
  else if (nm == "red_blocks") vec(P.red_blocks);
  else if (nm.size() > 6 && nm.compare(nm.size() - 6, 6, "_start") == 0) {  // gather lists, e.g. "gRed_start"
    const std::string gl = nm.substr(0, nm.size() - 6);
    const GatherList* G = gl == "gD" ? &P.gD : gl == "gE" ? &P.gE : gl == "gGp" ? &P.gGp : gl == "gW" ? &P.gW
                        : gl == "gRed" ? &P.gRed : gl == "gGred" ? &P.gGred : nullptr;
    if (!G) return DYNOHIP_EINVAL;
    raw(G->start.data(), G->start.size() * sizeof(int64_t));
  } else if (nm.size() > 4 && nm.compare(nm.size() - 4, 4, "_ent") == 0) {
    const std::string gl = nm.substr(0, nm.size() - 4);
    const GatherList* G = gl == "gD" ? &P.gD : gl == "gE" ? &P.gE : gl == "gGp" ? &P.gGp : gl == "gW" ? &P.gW
                        : gl == "gRed" ? &P.gRed : gl == "gGred" ? &P.gGred : nullptr;
    if (!G) return DYNOHIP_EINVAL;
    raw(G->ent.data(), G->ent.size() * sizeof(GEntry));
  }
  else if (nm == "red_b") vec(P.red_B);
  // lone-point groups (plan.hpp LoneGroup): the device blocks, each group's
  // (m, npt, pose_beg, out), its neighbour poses, the edge structure and the
  // PoseToPoint records they point into
  else if (nm == "lone_blk") raw(P.lone_blk.data(), P.lone_blk.size() * sizeof(int32_t));
  else if (nm == "lgroup") raw(P.lgroup.data(), P.lgroup.size() * sizeof(LoneGroup));
  else if (nm == "lone_pose") vec(P.lone_pose);
  else if (nm == "lone_info") {
    int32_t c_long = 0;
    while (c_long < P.n_comp && P.comp_start[c_long + 1] - P.comp_start[c_long] >= 2) ++c_long;
    tmp = {P.lone_all_grouped ? 1 : 0, static_cast<int32_t>(P.lgroup.size()), P.lone_max_m,
           c_long < P.n_comp ? P.comp_start[c_long] : P.n_pt, P.n_pt};
    vec(tmp);
  } else if (nm == "pt_edges") vec(P.pt_edge_start);   // (names ending in _start are gather lists)
  else if (nm == "edge_pose") vec(P.edge_pose);
  else if (nm == "comp_starts") vec(P.comp_start);
  else if (nm.size() == 9 && nm.compare(0, 8, "type_idx") == 0 && nm[8] >= '0' && nm[8] < '0' + kNTypes)
    vec(P.types[nm[8] - '0'].idx);
  else if (nm == "type_rec") {   // per type: arena offset of the first record, doubles per record
    for (int t = 0; t < kNTypes; ++t) {
      tmp.push_back(static_cast<int32_t>(P.types[t].base));
      tmp.push_back(static_cast<int32_t>(P.types[t].stride));
    }
    vec(tmp);
  }
  else if (nm == "digest") {
    // FNV-1a of every plan array and scalar, one 64-bit digest per field as
    // two int32 (tests/test_plan_digest.py: a plan built on one planner
    // worker equals the plan built on many, field by field)
    auto fnv = [&](const void* p, size_t bytes) {
      uint64_t h = 1469598103934665603ull;
      const auto* b = static_cast<const unsigned char*>(p);
      for (size_t i = 0; i < bytes; ++i) h = (h ^ b[i]) * 1099511628211ull;
      tmp.push_back(static_cast<int32_t>(h & 0xffffffffu));
      tmp.push_back(static_cast<int32_t>(h >> 32));
    };
    auto v = [&](const auto& x) { fnv(x.data(), x.size() * sizeof(x[0])); };
    const int64_t sc[] = {P.n_pose, P.n_pt, P.n_comp, P.max_chain, P.n_edge, P.lone_max_m, P.lone_all_grouped,
                          static_cast<int64_t>(P.off_I6), static_cast<int64_t>(P.off_D), static_cast<int64_t>(P.off_E),
                          static_cast<int64_t>(P.off_gp), static_cast<int64_t>(P.off_W), static_cast<int64_t>(P.off_Y),
                          static_cast<int64_t>(P.off_v), static_cast<int64_t>(P.off_L), static_cast<int64_t>(P.off_M),
                          static_cast<int64_t>(P.arena_size), P.n_red, P.NT, P.max_D, P.nd_leaf, P.n_slots,
                          P.n_partials};
    fnv(sc, sizeof(sc));
    v(P.user_kind); v(P.user_idx); v(P.pose_key); v(P.pt_key);
    v(P.comp_start); v(P.comp_nb_start); v(P.nb_pose); v(P.nb_comp); v(P.comp_y_base);
    v(P.nbedge_start); v(P.nbedge_pt); v(P.nbedge_w);
    v(P.edge_pt); v(P.edge_pose); v(P.pt_edge_start);
    for (int t = 0; t < kNTypes; ++t) {
      const int64_t ts[] = {P.types[t].n, static_cast<int64_t>(P.types[t].base), P.types[t].stride};
      fnv(ts, sizeof(ts));
      v(P.types[t].idx); v(P.types[t].meas); v(P.types[t].isig); v(P.types[t].hk);
    }
    for (const GatherList* G : {&P.gD, &P.gE, &P.gGp, &P.gW, &P.gRed, &P.gGred}) { v(G->start); v(G->ent); }
    v(P.red_A); v(P.red_B); v(P.red_slot); v(P.red_order); v(P.red_blocks);
    v(P.lgroup); v(P.lone_pose); v(P.lone_blk); v(P.lin_list0);
    v(P.band_D); v(P.tile_pos); v(P.row_start); v(P.row_col); v(P.row_slot);
    v(P.ftask); v(P.pairs); v(P.flevel); v(P.fpanels); v(P.fdep_start); v(P.fdep); v(P.fqueue);
    v(P.btask); v(P.blevel); v(P.bent); v(P.bpart); v(P.bplevel);
    v(P.tile_owner); v(P.sep_nodes); v(P.rhs0_tile); v(P.rhs0_start); v(P.rhs0_slot);
    for (const PartPhase& F : P.phases) {
      const int32_t hd[] = {F.node, F.leader};
      fnv(hd, sizeof(hd));
      v(F.xslot); v(F.xtile); v(F.ftask); v(F.flevel); v(F.fpanels); v(F.fdep_start); v(F.fdep); v(F.fqueue);
      v(F.rhs_tile); v(F.rhs_start); v(F.rhs_slot);
    }
    v(part.value_owner); v(part.damp_row);
    vec(tmp);
  }
  else if (nm == "value_owner") vec(part.value_owner);
  else if (nm == "damp_row") {
    tmp.assign(part.damp_row.begin(), part.damp_row.end());
    vec(tmp);
  } else return DYNOHIP_EINVAL;
  *n_out = cnt;
  if (out && cnt) std::memcpy(out, src, std::min(cap, cnt) * 4);
  return DYNOHIP_OK;
}
