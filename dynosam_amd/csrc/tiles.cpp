// tiles.cpp — tile-level symbolic factorisation and task schedule of the
// reduced pose system.
//
// The reference factors the reduced system inside GTSAM's multifrontal
// Cholesky. It eliminates the whole graph under a COLAMD ordering on every
// LM iteration (NonlinearOptimizer.cpp / GaussianFactorGraph::optimize,
// reached from RGBDBackendModule.cc:220 and :374).
//
// Here the points are removed analytically by the chain Schur complement,
// so the remaining pose system is a banded matrix over frame order. It is
// partitioned into 64x64 FP64 tiles, and its Cholesky is a DAG of two
// workgroup task kinds (tilechol.hip):
//   panel(k, i)    factor the diagonal tile A(k,k) (every panel of column k
//                  redundantly, in registers), then produce L(i,k). Before
//                  that it applies the last outstanding update of A(k,k) and
//                  of A(i,k). It also carries the forward substitution:
//                  y_k = L_kk^-1 r_k, then r_i -= L(i,k) y_k.
//   update(i,j,c)  A(i,j) -= L(i,c) L(j,c)^T.
// Tiles are ordered by nested dissection over frame order: recursive
// bisection of the tile range with a separator of the band's reach. Every
// leaf segment of the time axis is factored concurrently, and the
// separators are eliminated last. The DAG is scheduled in levels (longest
// path from the sources); one kernel launch runs one level. Natural order
// (no dissection) reproduces the plain band algorithm, one column per
// level. The leaf size is picked by a small cost model of the launch
// sequence.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <cstdint>
#include <functional>
#include <thread>
#include <vector>

#include "plan.hpp"
#include "plan_pool.hpp"

namespace dynohip {

namespace {

struct Sched {
  int leaf = 0;
  std::vector<int32_t> order;               // tile at position p
  std::vector<int32_t> pos;                 // position of tile t
  std::vector<int32_t> owner;               // per position: rank subtree, or sep_code(node) (partitioned)
  std::vector<int32_t> task_owner;          // per forward task: its rank, or the separator node it belongs to
  std::vector<SepNode> nodes;               // partitioned: the separator nodes of the top splits
  bool ok = true;                           // partitioned: every top split succeeded
  std::vector<std::vector<int32_t>> st;     // per column position: row positions (sorted, incl. itself)
  std::vector<int32_t> slot_base;           // per column position
  int32_t n_slots = 0;
  std::vector<TileTask> ftask;
  std::vector<int32_t> flevel;
  std::vector<int32_t> fpanels;
  std::vector<int32_t> pairs;
  std::vector<BackTask> btask;
  std::vector<int32_t> blevel;
  std::vector<int32_t> bent;
  double cost = 0.0;
  double flops = 0.0;

  int32_t slot(int rp, int cp) const {
    const auto& s = st[cp];
    const auto it = std::lower_bound(s.begin(), s.end(), rp);
    return slot_base[cp] + static_cast<int32_t>(it - s.begin());
  }
};

// nested-dissection order of tiles [lo, hi); maxnb[t] = largest neighbour
void nd_order(int lo, int hi, int leaf, const std::vector<int32_t>& maxnb, std::vector<int32_t>& out) {
  const int n = hi - lo;
  if (leaf <= 0 || n <= leaf) {
    for (int t = lo; t < hi; ++t) out.push_back(t);
    return;
  }
  const int m = lo + n / 2;
  int reach = m - 1;
  for (int t = lo; t < m; ++t) reach = std::max(reach, std::min(maxnb[t], hi - 1));
  const int s_end = reach + 1;  // separator [m, s_end)
  if (hi - s_end < 1 || s_end - m >= n / 2) {
    for (int t = lo; t < hi; ++t) out.push_back(t);
    return;
  }
  nd_order(lo, m, leaf, maxnb, out);
  nd_order(s_end, hi, leaf, maxnb, out);
  for (int t = m; t < s_end; ++t) out.push_back(t);
}

// Partitioned form: the top log2(nranks) levels of
// the dissection always split, and rank r owns the r-th leaf subtree in time
// order (its interior); the separators above them are owned by no rank (-1).
// A split of [lo, hi) over nr ranks (nl = nr / 2 on the left) is placed
// where the estimated factorisation work per rank of the two sides is most
// even: tile t's column weighs (env_t - t + 1)^2, env_t the largest
// neighbour of any tile up to t inside the range (the envelope a column's
// fill stays in; a banded column's Cholesky work grows with the square of
// its reach), so a graph denser in some stretch of time (objects
// visible for part of the sequence, configs[4]) does not leave one rank with
// most of the work. Fails (returns false) when a required split is
// impossible: the graph is too short in time for that many ranks; a
// balanced split that cannot be split further falls back to the midpoint.
bool part_split(int lo, int hi, const std::vector<int32_t>& maxnb, int nr, bool balanced, int& m_out,
                int& s_out) {
  const int n = hi - lo;
  if (n < 3) return false;
  const int nl = nr / 2;
  auto sep_end = [&](int m) {   // separator [m, s_end) of a split at m
    int reach = m - 1;
    for (int t = lo; t < m; ++t) reach = std::max(reach, std::min(maxnb[t], hi - 1));
    return reach + 1;
  };
  int m = lo + n / 2;
  if (balanced) {
    std::vector<double> wp(static_cast<size_t>(n) + 1, 0.0);   // prefix work
    int env = lo;   // the envelope: rows a column can fill down to
    for (int t = lo; t < hi; ++t) {
      env = std::max(env, std::min(maxnb[t], hi - 1));
      const double r = env - t + 1;
      wp[t - lo + 1] = wp[t - lo] + r * r;
    }
    double best = -1.0, at_mid = -1.0;
    int bm = m;
    int reach = lo;   // running max over [lo, mm) of the clipped neighbour reach
    for (int mm = lo + 1; mm < hi - 1; ++mm) {
      reach = std::max(reach, std::min(maxnb[mm - 1], hi - 1));
      const int se = std::max(reach, mm - 1) + 1;
      if (se <= mm || hi - se < 1) continue;
      // each side's subtree must split again for its ranks (>= 3 tiles)
      if ((nl > 1 && mm - lo < 3) || (nr - nl > 1 && hi - se < 3)) continue;
      const double c = std::max((wp[mm - lo] - wp[0]) / nl, (wp[n] - wp[se - lo]) / (nr - nl));
      if (mm == m) at_mid = c;
      if (best < 0.0 || c < best) {
        best = c;
        bm = mm;
      }
    }
    // the estimate is rough: a graph of even density keeps the midpoint
    // (within 15 % of the best estimate, the exact schedules favour it)
    if (best >= 0.0 && (at_mid < 0.0 || best < 0.85 * at_mid)) m = bm;
  }
  const int s_end = sep_end(m);
  if (hi - s_end < 1 || s_end <= m) return false;
  m_out = m;
  s_out = s_end;
  return true;
}

// A split's separator is a node of the partition tree: the ranks [r0, r0 +
// nr) of the subtree it splits factor it (after the exchange of its depth),
// depth 1 the top one. Its tiles get owner sep_code(node); nodes are numbered
// in creation order (children first).
bool nd_order_part_b(int lo, int hi, int leaf, const std::vector<int32_t>& maxnb, int nr, int r0,
                     std::vector<int32_t>& out, std::vector<int32_t>& owner, bool balanced,
                     std::vector<SepNode>& nodes, int depth) {
  if (nr == 1) {
    nd_order(lo, hi, leaf, maxnb, out);
    owner.resize(out.size(), r0);
    return true;
  }
  int m = 0, s_end = 0;
  if (!part_split(lo, hi, maxnb, nr, balanced, m, s_end)) return false;
  const int nl = nr / 2;
  const size_t o0 = out.size(), n0 = nodes.size();
  if (!nd_order_part_b(lo, m, leaf, maxnb, nl, r0, out, owner, balanced, nodes, depth + 1) ||
      !nd_order_part_b(s_end, hi, leaf, maxnb, nr - nl, r0 + nl, out, owner, balanced, nodes, depth + 1)) {
    out.resize(o0);
    owner.resize(o0);
    nodes.resize(n0);
    // the balanced split left a side that cannot split again: the midpoint
    return balanced && nd_order_part_b(lo, hi, leaf, maxnb, nr, r0, out, owner, false, nodes, depth);
  }
  const int32_t code = sep_code(static_cast<int32_t>(nodes.size()));
  nodes.push_back({r0, nr, depth, m, s_end});
  for (int t = m; t < s_end; ++t) {
    out.push_back(t);
    owner.push_back(code);
  }
  return true;
}

bool nd_order_part(int lo, int hi, int leaf, const std::vector<int32_t>& maxnb, int nr, int r0,
                   std::vector<int32_t>& out, std::vector<int32_t>& owner, std::vector<SepNode>& nodes) {
  static const bool balanced = [] {
    const char* e = std::getenv("DYNOHIP_PART_BALANCE");   // 0: split at the midpoint tile (round 3)
    return !(e && e[0] == '0');
  }();
  nodes.clear();
  return nd_order_part_b(lo, hi, leaf, maxnb, nr, r0, out, owner, balanced, nodes, 1);
}

constexpr int kUpdGroupTiles = 128;   // systems of this many tiles and more group update levels

void schedule(int NT, const std::vector<std::vector<int32_t>>& adj, const std::vector<int32_t>& maxnb, int leaf,
              Sched& S, int nranks = 1) {
  // levels of contributions per update task: large systems are throughput-
  // bound in the dataflow launch (NS: 11.5k update tasks, a top-separator
  // tile's chain of 22 one-level updates on the critical path), where two
  // levels per task measured best (NS factorisation 0.809 -> 0.740 ms;
  // 3: 0.745, 4: 0.747, 6: 0.805); small ones are latency-bound and keep one
  // (C2: 1: 0.289, 2: 0.291, 3: 0.297 ms). DYNOHIP_UPD_GROUP overrides.
  static const int32_t upd_env = [] {
    const char* e = std::getenv("DYNOHIP_UPD_GROUP");
    return e ? std::max(1, std::atoi(e)) : 0;
  }();
  const int32_t upd_group = upd_env > 0 ? upd_env : (NT >= kUpdGroupTiles ? 2 : 1);
  S.leaf = leaf;
  S.order.clear();
  S.owner.clear();
  if (nranks > 1) {
    S.ok = nd_order_part(0, NT, leaf, maxnb, nranks, 0, S.order, S.owner, S.nodes);
    if (!S.ok) return;
  } else {
    nd_order(0, NT, leaf, maxnb, S.order);
    S.owner.assign(NT, 0);
  }
  S.pos.assign(NT, 0);
  for (int p = 0; p < NT; ++p) S.pos[S.order[p]] = p;
  auto tm0 = std::chrono::steady_clock::now();
  auto tmark = [&](const char* what) {
    static const bool on = std::getenv("DYNOHIP_SCHED_TIMING") != nullptr;
    const auto t = std::chrono::steady_clock::now();
    if (on) std::fprintf(stderr, "  [sched leaf %d] %-24s %8.2f ms\n", leaf, what, std::chrono::duration<double, std::milli>(t - tm0).count());
    tm0 = t;
  };
  // ---- symbolic factorisation (elimination tree merge) in position space
  S.st.assign(NT, {});
  for (int cp = 0; cp < NT; ++cp) {
    auto& s = S.st[cp];
    s.push_back(cp);
    for (int32_t u : adj[S.order[cp]]) {
      const int up = S.pos[u];
      if (up > cp) s.push_back(up);
    }
  }
  for (int cp = 0; cp < NT; ++cp) {
    auto& s = S.st[cp];
    std::sort(s.begin(), s.end());
    s.erase(std::unique(s.begin(), s.end()), s.end());
    if (s.size() > 1) {
      auto& par = S.st[s[1]];
      par.insert(par.end(), s.begin() + 1, s.end());
    }
  }
  S.slot_base.assign(NT, 0);
  int32_t ns = 0;
  for (int cp = 0; cp < NT; ++cp) {
    S.slot_base[cp] = ns;
    ns += static_cast<int32_t>(S.st[cp].size());
  }
  S.n_slots = ns;
  tmark("symbolic");
  // ---- tasks with levels (1-based; 0 = available at start). Every stored
  // tile collects its update contributions (column c, ready level R_c).
  // Contributions ready one level before the tile's panel are applied by
  // the panel itself; earlier ones by update tasks. Each update task applies
  // every contribution ready by then, so a tile's read-modify-write chain
  // is as long as the number of distinct ready levels, not the number of
  // columns.
  struct Contrib {
    int32_t R, a, b;  // ready level, operand slots (A B^T)
    int32_t own;      // owner of the source column
  };
  // every slot's contributions in generation (column) order, in one pool
  // laid out by slot (counted first: a column adds one contribution to each
  // slot (s[x], s[y]), x >= y >= 1, of its structure), and the largest ready
  // level. The slot of (s[x], s[y]) is found by walking column s[y]'s
  // structure, which holds every s[x] (fill-path theorem), in step with x.
  auto each_pair_slot = [&](const std::vector<int32_t>& s, auto&& fn) {   // fn(x, y, slot)
    for (size_t y = 1; y < s.size(); ++y) {
      const auto& sy = S.st[s[y]];
      const int32_t base = S.slot_base[s[y]];
      size_t pos = 0;
      for (size_t x = y; x < s.size(); ++x) {
        while (sy[pos] < s[x]) ++pos;
        fn(x, y, base + static_cast<int32_t>(pos));
      }
    }
  };
  std::vector<int64_t> cstart(static_cast<size_t>(ns) + 1, 0);
  for (int cp = 0; cp < NT; ++cp) each_pair_slot(S.st[cp], [&](size_t, size_t, int32_t sl) { cstart[sl + 1]++; });
  for (int32_t sl = 0; sl < ns; ++sl) cstart[sl + 1] += cstart[sl];
  std::vector<Contrib> cpool(cstart[ns]);
  std::vector<int64_t> cfill(cstart.begin(), cstart.end() - 1);
  std::vector<int32_t> cmaxR(ns, 0);
  auto add_contrib = [&](int32_t sl, const Contrib& c) {
    cpool[cfill[sl]++] = c;
    cmaxR[sl] = std::max(cmaxR[sl], c.R);
  };
  std::vector<int32_t> lvlP(ns, 0);
  // a task; its operand pairs are ranges of one pool (a column's panels
  // share their diagonal tile's pending pairs)
  struct LT {
    int32_t lvl;
    TileTask t;
    int32_t pd_off, pd_n, po_off, po_n;  // pairs [off, off + n) of ppool (in pairs)
    int32_t own;                          // rank running the task (-1: after the exchange)
  };
  std::vector<LT> tasks;
  std::vector<int32_t> ppool;   // 2 ints per pair
  // every contribution becomes one pair (of an update or of the panel that
  // absorbs it); a slot has one panel and at most one update per ready level
  ppool.reserve(2 * cpool.size());
  tasks.reserve(2 * static_cast<size_t>(ns));
  const double T3 = static_cast<double>(kTile) * kTile * kTile;
  double flops = 0.0;
  std::vector<Contrib> all, cs, mine;
  std::vector<int32_t> owners;
  auto pool_pairs = [&]() { return static_cast<int32_t>(ppool.size() / 2); };
  // split contributions (sorted by R) into update tasks finishing before
  // level P and the pairs the panel at level P absorbs (appended to ppool
  // last: [*aoff, *aoff + *an))
  // Partitioned: a separator tile takes the contributions of every column
  // outside its own node (interior columns, deeper separators) as update
  // tasks of the source column's owner, never absorbed by its panel, so that
  // the tile holds partial sums per rank until its node's exchange.
  auto plan_tile = [&](int32_t sl, int32_t P, int32_t* aoff, int32_t* an, int32_t town) {
    all.assign(cpool.begin() + cstart[sl], cpool.begin() + cfill[sl]);
    std::sort(all.begin(), all.end(), [](const Contrib& x, const Contrib& y) { return x.R < y.R; });
    // an update task takes the contributions ready within upd_group levels
    // of its first one (1: one task per distinct ready level), so a tile fed
    // at many levels has a shorter read-modify-write chain of update tasks
    auto emit_updates = [&](const std::vector<Contrib>& v, size_t& q, int32_t limitR, int32_t own) {
      while (q < v.size() && v[q].R <= limitR) {
        const int32_t last = std::min(limitR, v[q].R + upd_group - 1);
        LT u{0, TileTask{1, -1, -1, sl, -1, 0, 0, 0, 0, 0}, 0, 0, pool_pairs(), 0, own};
        int32_t rmax = v[q].R;
        while (q < v.size() && v[q].R <= last) {
          rmax = std::max(rmax, v[q].R);
          ppool.push_back(v[q].a);
          ppool.push_back(v[q].b);
          ++q;
        }
        u.lvl = rmax + 1;
        u.po_n = pool_pairs() - u.po_off;
        tasks.push_back(u);
      }
    };
    cs.clear();
    if (town < 0) {
      owners.clear();
      for (const Contrib& c : all)
        if (c.own != town) owners.push_back(c.own);
      std::sort(owners.begin(), owners.end());
      owners.erase(std::unique(owners.begin(), owners.end()), owners.end());
      for (int32_t o : owners) {
        size_t q = 0;
        mine.clear();
        for (const Contrib& c : all)
          if (c.own == o) mine.push_back(c);
        emit_updates(mine, q, INT32_MAX, o);
      }
      for (const Contrib& c : all)
        if (c.own == town) cs.push_back(c);
    } else {
      cs = all;
    }
    size_t q = 0;
    emit_updates(cs, q, P - 2, town);
    *aoff = pool_pairs();
    for (; q < cs.size(); ++q) {
      ppool.push_back(cs[q].a);
      ppool.push_back(cs[q].b);
    }
    *an = pool_pairs() - *aoff;
  };
  for (int cp = 0; cp < NT; ++cp) {
    const auto& s = S.st[cp];
    const int32_t dslot = S.slot_base[cp];   // s[0] == cp
    const int32_t Pd = cmaxR[dslot] + 1;
    const int32_t cown = S.owner[cp];
    int32_t pd_off = 0, pd_n = 0;
    plan_tile(dslot, Pd, &pd_off, &pd_n, cown);
    flops += T3 / 3.0;
    for (size_t x = 0; x < s.size(); ++x) {
      const int32_t rp = s[x];
      const int32_t sl = S.slot_base[cp] + static_cast<int32_t>(x);
      LT t{Pd, TileTask{0, S.order[cp], S.order[rp], sl, dslot, 0, 0, 0, 0, 0}, pd_off, pd_n, 0, 0, cown};
      if (rp != cp) {
        t.lvl = std::max(Pd, cmaxR[sl] + 1);
        plan_tile(sl, t.lvl, &t.po_off, &t.po_n, cown);
        flops += T3;
      }
      lvlP[sl] = t.lvl;
      tasks.push_back(t);
    }
    // (a slot receives at most one contribution per column, so the order of
    // the pairs within a column does not change any slot's list)
    each_pair_slot(s, [&](size_t x, size_t y, int32_t sl) {
      const int32_t sa = S.slot_base[cp] + static_cast<int32_t>(x), sb = S.slot_base[cp] + static_cast<int32_t>(y);
      add_contrib(sl, {std::max(lvlP[sa], lvlP[sb]), sa, sb, cown});
      flops += 2.0 * T3;
    });
  }
  S.flops = flops;
  tmark("contributions/tasks");
  // by level; within a level panels first, then updates (wide levels run
  // their updates as a separate, concurrent kernel): a stable counting sort
  int32_t maxlvl = 0;
  for (const LT& t : tasks) maxlvl = std::max(maxlvl, t.lvl);
  std::vector<int32_t> bstart(2 * (static_cast<size_t>(maxlvl) + 1) + 1, 0);
  for (const LT& t : tasks) bstart[2 * t.lvl + t.t.kind + 1]++;
  for (size_t k = 1; k < bstart.size(); ++k) bstart[k] += bstart[k - 1];
  std::vector<int32_t> perm(tasks.size());
  for (size_t q = 0; q < tasks.size(); ++q) perm[bstart[2 * tasks[q].lvl + tasks[q].t.kind]++] = static_cast<int32_t>(q);
  S.ftask.clear();
  S.flevel.clear();
  S.pairs.clear();
  S.task_owner.clear();
  S.ftask.reserve(tasks.size());
  S.task_owner.reserve(tasks.size());
  S.pairs.reserve(ppool.size());
  int cur = 0;
  for (int32_t qi : perm) {
    LT& t = tasks[qi];
    while (cur < t.lvl) {
      S.flevel.push_back(static_cast<int32_t>(S.ftask.size()));
      ++cur;
    }
    auto put = [&](int32_t off, int32_t n, int32_t& beg, int32_t& end) {
      beg = static_cast<int32_t>(S.pairs.size() / 2);
      S.pairs.insert(S.pairs.end(), ppool.begin() + 2 * off, ppool.begin() + 2 * (off + n));
      end = static_cast<int32_t>(S.pairs.size() / 2);
    };
    put(t.pd_off, t.pd_n, t.t.pd_beg, t.t.pd_end);
    put(t.po_off, t.po_n, t.t.po_beg, t.t.po_end);
    S.ftask.push_back(t.t);
    S.task_owner.push_back(t.own);
  }
  S.flevel.push_back(static_cast<int32_t>(S.ftask.size()));
  S.fpanels.assign(S.flevel.size() - 1, 0);
  for (size_t l = 0; l + 1 < S.flevel.size(); ++l)
    for (int32_t q = S.flevel[l]; q < S.flevel[l + 1]; ++q) S.fpanels[l] += S.ftask[q].kind == 0;
  tmark("sort/flatten");
  // ---- backward substitution levels
  std::vector<int32_t> blv(NT, 0);
  int maxb = 0;
  for (int cp = NT - 1; cp >= 0; --cp) {
    int32_t L = 0;
    for (size_t x = 1; x < S.st[cp].size(); ++x) L = std::max(L, blv[S.st[cp][x]]);
    blv[cp] = L + 1;
    maxb = std::max(maxb, L + 1);
  }
  S.btask.clear();
  S.blevel.assign(1, 0);
  S.bent.clear();
  for (int lv = 1; lv <= maxb; ++lv) {
    for (int cp = NT - 1; cp >= 0; --cp) {
      if (blv[cp] != lv) continue;
      BackTask b{S.order[cp], static_cast<int32_t>(S.bent.size() / 2), 0, 0};
      for (size_t x = 1; x < S.st[cp].size(); ++x) {
        S.bent.push_back(S.slot(S.st[cp][x], cp));
        S.bent.push_back(S.order[S.st[cp][x]]);
      }
      b.end = static_cast<int32_t>(S.bent.size() / 2);
      S.btask.push_back(b);
    }
    S.blevel.push_back(static_cast<int32_t>(S.btask.size()));
  }
  // ---- cost model (microseconds, calibrated with per-task clock64 stamps
  // on MI355X): a level costs its launch plus the longer of its longest task
  // and its total task time spread over the CUs (one 158 KB-LDS workgroup
  // per CU). A panel is ~24 us (dominated by the in-register diagonal
  // factorisation), an update ~5 us, plus ~1.7 us per operand pair (a 64^3
  // FP64 MFMA GEMM on one CU).
  constexpr int kCUs = 256;
  double cost = 0.0;
  const int nlev = static_cast<int>(S.flevel.size()) - 1;
  for (int l = 0; l < nlev; ++l) {
    double worst = 0.0, total = 0.0;
    for (int32_t q = S.flevel[l]; q < S.flevel[l + 1]; ++q) {
      const TileTask& t = S.ftask[q];
      const int np = (t.pd_end - t.pd_beg) + (t.po_end - t.po_beg);
      const double c = (t.kind == 0 ? 24.0 : 5.0) + 1.7 * np;
      worst = std::max(worst, c);
      total += c;
    }
    cost += 1.0 + std::max(worst, total / kCUs);
  }
  for (size_t l = 0; l + 1 < S.blevel.size(); ++l) cost += 4.0;
  S.cost = cost;
  tmark("backward/cost");
}

int g_leaf_override = -1;
// workgroups of the dataflow launch the queue order is simulated on (0:
// level order, the schedule's own order; DYNOHIP_QUEUE_ORDER=level, read at
// every plan build)
int queue_workers() {
  const char* e = std::getenv("DYNOHIP_QUEUE_ORDER");
  return (e && std::string(e) == "level") ? 0 : 256;
}

// Per task, the slots it reads or writes and how many writes each must have
// received first: the writes of earlier levels (the level schedule is a valid
// order, so this reproduces it exactly, including the fixed order in which a
// tile receives its updates). Slots only written before the factorisation
// (count 0) are left out.
void build_dataflow_deps(const Plan& P, const std::vector<TileTask>& ftask, const std::vector<int32_t>& flevel,
                         std::vector<int32_t>& fdep_start, std::vector<int32_t>& fdep) {
  std::vector<int32_t> written(P.n_slots, 0);
  fdep_start.assign(1, 0);
  fdep.clear();
  std::vector<int32_t> touch;
  const int nlev = static_cast<int>(flevel.size()) - 1;
  for (int l = 0; l < nlev; ++l) {
    for (int32_t q = flevel[l]; q < flevel[l + 1]; ++q) {
      const TileTask& t = ftask[q];
      touch.clear();
      auto add_pairs = [&](int32_t beg, int32_t end) {
        for (int32_t e = beg; e < end; ++e) {
          touch.push_back(P.pairs[2 * e]);
          touch.push_back(P.pairs[2 * e + 1]);
        }
      };
      add_pairs(t.po_beg, t.po_end);
      if (t.kind == 1) {
        touch.push_back(t.dst);
      } else {
        touch.push_back(t.diag);
        add_pairs(t.pd_beg, t.pd_end);
        if (t.i != t.k) touch.push_back(t.dst);
        for (int32_t e = P.row_start[t.k]; e < P.row_start[t.k + 1]; ++e)
          if (P.row_col[e] != t.k) touch.push_back(P.row_slot[e]);
      }
      std::sort(touch.begin(), touch.end());
      touch.erase(std::unique(touch.begin(), touch.end()), touch.end());
      for (int32_t sl : touch)
        if (written[sl] > 0) {
          fdep.push_back(sl);
          fdep.push_back(written[sl]);
        }
      fdep_start.push_back(static_cast<int32_t>(fdep.size() / 2));
    }
    for (int32_t q = flevel[l]; q < flevel[l + 1]; ++q) {
      const TileTask& t = ftask[q];
      if (t.kind == 1 || t.i != t.k) written[t.dst]++;
    }
  }
}

// The dataflow kernel's queue order. Workgroups take tasks in queue order
// and wait, holding their CU, until the task's inputs are written. In level
// order, a wide graph (NS: 14.6k tasks, 256 workgroups) fills every
// workgroup with tasks of later levels that wait while ready tasks queue
// behind them: 20 us of queueing per task on average, most of it on the
// critical path (tools/task_clock.py, profiles/r03/task_clock_NS.txt). The
// queue is therefore a list schedule of the dependency graph simulated on
// `workers` workgroups: a task is ready a hand-off after its inputs' writers
// end, among the ready tasks the one with the longest remaining path starts
// first (estimated costs below), and the queue lists tasks by simulated
// start. That is a topological order of the dependencies (each
// starts after its inputs' writers end), so the launch stays deadlock-free.
// estimated costs (us, MI355X task clock): a panel and an update task
// without operand pairs, a 64^3 operand pair, a write-to-reader hand-off
// (the NS rate moved < 0.5% over panel 16-20, update 5.5-11, hand-off 2.5-6)
// the queue order's cost model (us): a panel, an update, per pending pair, a
// hand-off. DYNOHIP_QCOST="panel,update,pair,handoff" overrides it (tuning).
struct QCost {
  double panel = 16.0, update = 5.5, pair = 1.7, handoff = 2.5;
};
const QCost& qcost() {
  static const QCost c = [] {
    QCost q;
    if (const char* e = std::getenv("DYNOHIP_QCOST"))
      std::sscanf(e, "%lf,%lf,%lf,%lf", &q.panel, &q.update, &q.pair, &q.handoff);
    return q;
  }();
  return c;
}
constexpr int kQueueSimMax = 100000;
std::vector<int32_t> queue_order(const Plan& P, const std::vector<TileTask>& ftask,
                                 const std::vector<int32_t>& flevel, const std::vector<int32_t>& fdep_start,
                                 const std::vector<int32_t>& fdep, int workers) {
  const int n = static_cast<int>(ftask.size());
  std::vector<int32_t> order(n);
  for (int q = 0; q < n; ++q) order[q] = q;
  // (above kQueueSimMax tasks the simulation's host time, ~0.7 us per task,
  // is not spent: C5's 538k tasks would add 0.37 s of planning, and the
  // one-GPU measurements that favour it are at NS, 14.6k tasks)
  if (n == 0 || workers <= 0 || n > kQueueSimMax) return order;
  std::vector<double> dur(n);
  for (int q = 0; q < n; ++q) {
    const TileTask& t = ftask[q];
    const int np = (t.pd_end - t.pd_beg) + (t.po_end - t.po_beg);
    dur[q] = (t.kind == 0 ? qcost().panel : qcost().update) + qcost().pair * np;
  }
  // predecessor lists (the writer of each awaited write, counted in level order)
  std::vector<int32_t> wcount(P.n_slots, 0), wstart(P.n_slots + 1, 0);
  for (int q = 0; q < n; ++q)
    if (ftask[q].kind == 1 || ftask[q].i != ftask[q].k) wstart[ftask[q].dst + 1]++;
  for (int sl = 0; sl < P.n_slots; ++sl) wstart[sl + 1] += wstart[sl];
  std::vector<int32_t> writer(wstart[P.n_slots]);
  const int nlev = static_cast<int>(flevel.size()) - 1;
  for (int l = 0; l < nlev; ++l)
    for (int32_t q = flevel[l]; q < flevel[l + 1]; ++q)
      if (ftask[q].kind == 1 || ftask[q].i != ftask[q].k) writer[wstart[ftask[q].dst] + wcount[ftask[q].dst]++] = q;
  std::vector<int32_t> npred(n, 0), sstart(n + 1, 0);
  for (int q = 0; q < n; ++q)
    for (int32_t j = fdep_start[q]; j < fdep_start[q + 1]; ++j) sstart[writer[wstart[fdep[2 * j]] + fdep[2 * j + 1] - 1] + 1]++;
  for (int q = 0; q < n; ++q) sstart[q + 1] += sstart[q];
  std::vector<int32_t> succ(sstart[n]), sfill(sstart.begin(), sstart.end() - 1);
  for (int q = 0; q < n; ++q)
    for (int32_t j = fdep_start[q]; j < fdep_start[q + 1]; ++j) {
      succ[sfill[writer[wstart[fdep[2 * j]] + fdep[2 * j + 1] - 1]]++] = q;
      npred[q]++;
    }
  // remaining path length, hand-offs included (tasks are in a topological
  // order already: levels)
  std::vector<double> rem(n, 0.0);
  for (int q = n - 1; q >= 0; --q) {
    double m = 0.0;
    for (int32_t j = sstart[q]; j < sstart[q + 1]; ++j) m = std::max(m, qcost().handoff + rem[succ[j]]);
    rem[q] = dur[q] + m;
  }
  // list scheduling: ready heap by remaining path; tasks whose inputs are
  // written wait out the hand-off in a heap by ready time; running heap by end
  auto by_rem = [&](int32_t a, int32_t b) { return rem[a] < rem[b] || (rem[a] == rem[b] && a > b); };
  using TQ = std::pair<double, int32_t>;
  auto later = [](const TQ& a, const TQ& b) { return a.first > b.first || (a.first == b.first && a.second > b.second); };
  std::vector<int32_t> ready;
  std::vector<TQ> running, pending;
  std::vector<double> start(n, 0.0), rdy(n, 0.0);
  for (int q = 0; q < n; ++q)
    if (npred[q] == 0) ready.push_back(q);
  std::make_heap(ready.begin(), ready.end(), by_rem);
  double now = 0.0;
  int free_w = std::max(1, workers), done = 0;
  while (done < n) {
    while (!pending.empty() && pending.front().first <= now) {
      std::pop_heap(pending.begin(), pending.end(), later);
      ready.push_back(pending.back().second);
      std::push_heap(ready.begin(), ready.end(), by_rem);
      pending.pop_back();
    }
    while (free_w > 0 && !ready.empty()) {
      std::pop_heap(ready.begin(), ready.end(), by_rem);
      const int32_t q = ready.back();
      ready.pop_back();
      start[q] = now;
      running.push_back({now + dur[q], q});
      std::push_heap(running.begin(), running.end(), later);
      --free_w;
    }
    // next event: a task ends or a hand-off completes
    const double t_end = running.empty() ? INFINITY : running.front().first;
    const double t_rdy = pending.empty() ? INFINITY : pending.front().first;
    if (!(std::min(t_end, t_rdy) < INFINITY)) break;   // (cannot happen: the graph is acyclic)
    if (t_rdy < t_end) {
      now = t_rdy;
      continue;
    }
    std::pop_heap(running.begin(), running.end(), later);
    const TQ fin = running.back();
    running.pop_back();
    now = fin.first;
    ++free_w;
    ++done;
    for (int32_t j = sstart[fin.second]; j < sstart[fin.second + 1]; ++j) {
      const int32_t sq = succ[j];
      rdy[sq] = std::max(rdy[sq], now + qcost().handoff);
      if (--npred[sq] == 0) {
        pending.push_back({rdy[sq], sq});
        std::push_heap(pending.begin(), pending.end(), later);
      }
    }
  }
  std::stable_sort(order.begin(), order.end(), [&](int32_t a, int32_t b) { return start[a] < start[b]; });
  return order;
}

// keep the tasks q with keep(q), in schedule order, with their levels
// renumbered densely (empty levels dropped)
template <class Keep>
void filter_tasks(const std::vector<TileTask>& all, const std::vector<int32_t>& lev, Keep&& keep,
                  std::vector<TileTask>& ftask, std::vector<int32_t>& flevel, std::vector<int32_t>& fpanels) {
  ftask.clear();
  flevel.assign(1, 0);
  fpanels.clear();
  for (size_t l = 0; l + 1 < lev.size(); ++l) {
    int np = 0;
    for (int32_t q = lev[l]; q < lev[l + 1]; ++q)
      if (keep(q)) {
        ftask.push_back(all[q]);
        np += all[q].kind == 0;
      }
    if (static_cast<int32_t>(ftask.size()) != flevel.back()) {
      flevel.push_back(static_cast<int32_t>(ftask.size()));
      fpanels.push_back(np);
    }
  }
}

// largest tile each tile shares a reduced block with (at least itself)
std::vector<int32_t> tile_maxnb(const Plan& P) {
  std::vector<int32_t> maxnb(P.NT);
  for (int t = 0; t < P.NT; ++t) maxnb[t] = t;
  for (size_t q = 0; q < P.red_A.size(); ++q) {
    const int r1 = (6 * P.red_A[q] + 5) / kTile;
    const int c0 = (6 * P.red_B[q]) / kTile;
    // the pair's tiles span rows r0..r1 and columns c0..c1; the smallest
    // tile of any cross pair is >= c0 and the largest <= r1
    maxnb[c0] = std::max(maxnb[c0], r1);
    const int c1 = (6 * P.red_B[q] + 5) / kTile, r0 = (6 * P.red_A[q]) / kTile;
    for (int a = r0; a <= r1; ++a)
      for (int b = c0; b <= c1; ++b)
        if (a != b) maxnb[std::min(a, b)] = std::max(maxnb[std::min(a, b)], std::max(a, b));
  }
  return maxnb;
}

}  // namespace

// the tile owners of nd_order_part's top splits (in natural tile order)
bool partition_tile_owners(const Plan& P, int nranks, std::vector<int32_t>& owner, std::vector<SepNode>& nodes) {
  owner.assign(P.NT, 0);
  nodes.clear();
  if (nranks <= 1) return true;
  std::vector<int32_t> out, own;
  if (!nd_order_part(0, P.NT, 0, tile_maxnb(P), nranks, 0, out, own, nodes)) return false;
  for (size_t q = 0; q < out.size(); ++q) owner[out[q]] = own[q];
  return true;
}

bool build_tile_schedule(Plan& P, bool own_threads) {
  const int NT = P.NT;
  auto bt0 = std::chrono::steady_clock::now();
  auto bmark = [&](const char* what) {
    static const bool on = std::getenv("DYNOHIP_SCHED_TIMING") != nullptr;
    const auto t = std::chrono::steady_clock::now();
    if (on) std::fprintf(stderr, "  [tiles] %-28s %8.2f ms\n", what, std::chrono::duration<double, std::milli>(t - bt0).count());
    bt0 = t;
  };
  std::vector<std::vector<int32_t>> adj(NT);
  std::vector<int32_t> maxnb(NT);
  for (int t = 0; t < NT; ++t) maxnb[t] = t;
  for (size_t q = 0; q < P.red_A.size(); ++q) {
    const int r0 = (6 * P.red_A[q]) / kTile, r1 = (6 * P.red_A[q] + 5) / kTile;
    const int c0 = (6 * P.red_B[q]) / kTile, c1 = (6 * P.red_B[q] + 5) / kTile;
    for (int a = r0; a <= r1; ++a)
      for (int b = c0; b <= c1; ++b) {
        if (a == b) continue;
        adj[a].push_back(b);
        adj[b].push_back(a);
        maxnb[std::min(a, b)] = std::max(maxnb[std::min(a, b)], std::max(a, b));
      }
  }
  for (auto& v : adj) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
  }
  const int nr = std::max(1, P.nranks);
  bmark("adjacency");
  Sched best;
  if (g_leaf_override >= 0) {
    schedule(NT, adj, maxnb, g_leaf_override, best, nr);
    if (!best.ok) return false;
  } else {
    // frame order (leaf 0) and the nested-dissection leaf sizes are
    // independent schedules: built on threads, then the cheapest kept in
    // list order, frame order first (the same choice as a serial scan).
    // Leaves below 16 tiles are not candidates of large systems: the cost
    // model never picks them there, and their deep dissections are the
    // costliest schedules to build.
    std::vector<int> leaves{0};
    for (int leaf : {4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256}) {
      if (leaf * nr >= NT) break;
      if (NT > 512 && leaf < 16) continue;
      leaves.push_back(leaf);
    }
    std::vector<Sched> cand(leaves.size());
    if (own_threads) {
      std::vector<std::thread> th;
      for (size_t c = 1; c < leaves.size(); ++c)
        th.emplace_back([&, c] { schedule(NT, adj, maxnb, leaves[c], cand[c], nr); });
      schedule(NT, adj, maxnb, leaves[0], cand[0], nr);
      for (auto& t : th) t.join();
    } else {
      parallel_chunks(static_cast<int64_t>(leaves.size()), 1, [&](int64_t c0, int64_t c1) {
        for (int64_t c = c0; c < c1; ++c) schedule(NT, adj, maxnb, leaves[c], cand[c], nr);
      });
    }
    if (!cand[0].ok) return false;
    size_t bi = 0;
    for (size_t c = 1; c < cand.size(); ++c)
      if (cand[c].ok && cand[c].cost < cand[bi].cost) bi = c;
    best = std::move(cand[bi]);
  }
  bmark("schedules");
  P.nd_leaf = best.leaf;
  P.tile_pos = best.pos;
  P.n_slots = best.n_slots;
  P.tile_flops = best.flops;
  P.ftask = std::move(best.ftask);
  P.pairs = std::move(best.pairs);
  P.flevel = std::move(best.flevel);
  P.fpanels = std::move(best.fpanels);
  P.btask = std::move(best.btask);
  P.blevel = std::move(best.blevel);
  P.bent = std::move(best.bent);
  // split every backward task into workgroups of <= back_part_tiles entries:
  // the smallest power of two (>= 4: the tiles a part holds in registers
  // before its wait) whose part count lets the one-launch backward solve
  // keep every workgroup resident
  auto count_parts = [&](int tpp) {
    int64_t n = 0;
    for (const BackTask& t : P.btask) n += std::max<int32_t>(1, (t.end - t.beg + tpp - 1) / tpp);
    return n;
  };
  P.back_part_tiles = 4;
  if (const char* e = std::getenv("DYNOHIP_BACK_PART_TILES")) P.back_part_tiles = std::max(1, std::atoi(e));   // sweep knob
  while (count_parts(P.back_part_tiles) > kBackPersistMax && P.back_part_tiles < 64) P.back_part_tiles *= 2;
  if (count_parts(P.back_part_tiles) > kBackPersistMax) P.back_part_tiles = 4;  // level launches
  const int32_t tpp = P.back_part_tiles;
  P.bpart.clear();
  P.bplevel.assign(1, 0);
  P.n_partials = 0;
  for (size_t l = 0; l + 1 < P.blevel.size(); ++l) {
    for (int32_t q = P.blevel[l]; q < P.blevel[l + 1]; ++q) {
      const BackTask& t = P.btask[q];
      const int32_t n = t.end - t.beg;
      const int32_t np = std::max<int32_t>(1, (n + tpp - 1) / tpp);
      const int32_t pbase = np > 1 ? P.n_partials : -1;
      if (np > 1) P.n_partials += np;
      for (int32_t part = 0; part < np; ++part) {
        const int32_t b0 = t.beg + part * tpp;
        P.bpart.push_back({t.k, b0, std::min(t.end, b0 + tpp), np, part, pbase, 0, 0});
      }
    }
    P.bplevel.push_back(static_cast<int32_t>(P.bpart.size()));
  }
  bmark("backward parts");
  // per-row lookup for the assembly: stored tile (row tile, column tile)
  std::vector<std::vector<std::pair<int32_t, int32_t>>> rows(NT);
  for (int cp = 0; cp < NT; ++cp)
    for (int32_t rp : best.st[cp]) rows[best.order[rp]].push_back({best.order[cp], best.slot(rp, cp)});
  P.row_start.assign(NT + 1, 0);
  P.row_col.clear();
  P.row_slot.clear();
  for (int t = 0; t < NT; ++t) {
    std::sort(rows[t].begin(), rows[t].end());
    for (const auto& e : rows[t]) {
      P.row_col.push_back(e.first);
      P.row_slot.push_back(e.second);
    }
    P.row_start[t + 1] = static_cast<int32_t>(P.row_col.size());
  }
  // ---- partitioned: this rank's phase-0 tasks (its subtree, and its
  // interior columns' updates of separator tiles), then one phase per
  // separator node on its path to the top, deepest first. A node's phase
  // runs on every rank of its group: its panels and the updates among its
  // own tiles; its updates of the separators above it run on the group's
  // leader only (the others' copies of those tiles keep their own partial
  // sums, so the next exchange counts each contribution once).
  P.tile_owner.assign(NT, 0);
  for (int cp = 0; cp < NT; ++cp) P.tile_owner[best.order[cp]] = best.owner[cp];
  P.sep_nodes = best.nodes;
  P.phases.clear();
  P.rhs0_tile.clear();
  P.rhs0_start.assign(1, 0);
  P.rhs0_slot.clear();
  if (nr > 1) {
    const std::vector<TileTask> all = P.ftask;
    const std::vector<int32_t> lev = P.flevel;
    // the owner of each slot's column
    std::vector<int32_t> slot_own(best.n_slots);
    for (int cp = 0; cp < NT; ++cp)
      for (size_t x = 0; x < best.st[cp].size(); ++x) slot_own[best.slot_base[cp] + x] = best.owner[cp];
    auto in_group = [&](int32_t node, int32_t r) {
      const SepNode& nd = P.sep_nodes[node];
      return r >= nd.r0 && r < nd.r0 + nd.nr;
    };
    filter_tasks(all, lev, [&](int32_t q) { return best.task_owner[q] == P.rank; }, P.ftask, P.flevel, P.fpanels);
    // this rank's nodes, deepest first
    std::vector<int32_t> path;
    for (int32_t nd = 0; nd < static_cast<int32_t>(P.sep_nodes.size()); ++nd)
      if (in_group(nd, P.rank)) path.push_back(nd);
    std::stable_sort(path.begin(), path.end(),
                     [&](int32_t a, int32_t b) { return P.sep_nodes[a].depth > P.sep_nodes[b].depth; });
    // slot ranges of a node's columns (contiguous per column position)
    auto node_slots = [&](int32_t depth, std::vector<int32_t>& xs, std::vector<int32_t>& xt) {
      xs.clear();
      xt.clear();
      for (int cp = 0; cp < NT; ++cp) {
        const int32_t o = best.owner[cp];
        if (o >= 0 || P.sep_nodes[sep_node(o)].depth != depth) continue;
        const int32_t b = best.slot_base[cp], e = b + static_cast<int32_t>(best.st[cp].size());
        if (!xs.empty() && xs.back() == b) xs.back() = e;
        else {
          xs.push_back(b);
          xs.push_back(e);
        }
      }
      for (int t = 0; t < NT; ++t) {
        const int32_t o = P.tile_owner[t];
        if (o >= 0 || P.sep_nodes[sep_node(o)].depth != depth) continue;
        if (!xt.empty() && xt.back() == t) xt.back() = t + 1;
        else {
          xt.push_back(t);
          xt.push_back(t + 1);
        }
      }
    };
    // the contributions of columns owned by `src` to rows of other
    // separators (k_sep_rhs lists)
    auto rhs_lists = [&](int32_t src, std::vector<int32_t>& tl, std::vector<int32_t>& ts, std::vector<int32_t>& sl) {
      tl.clear();
      ts.assign(1, 0);
      sl.clear();
      for (int t = 0; t < NT; ++t) {
        const int32_t o = P.tile_owner[t];
        if (o >= 0 || o == src) continue;
        const size_t n0 = sl.size();
        for (int32_t e = P.row_start[t]; e < P.row_start[t + 1]; ++e)
          if (P.tile_owner[P.row_col[e]] == src) sl.push_back(P.row_slot[e]);
        if (sl.size() == n0) continue;
        tl.push_back(t);
        ts.push_back(static_cast<int32_t>(sl.size()));
      }
    };
    rhs_lists(P.rank, P.rhs0_tile, P.rhs0_start, P.rhs0_slot);
    P.phases.resize(path.size());
    for (size_t ph = 0; ph < path.size(); ++ph) {
      PartPhase& F = P.phases[ph];
      const int32_t nd = path[ph], code = sep_code(nd);
      F.node = nd;
      F.leader = P.sep_nodes[nd].r0 == P.rank ? 1 : 0;
      node_slots(P.sep_nodes[nd].depth, F.xslot, F.xtile);
      filter_tasks(all, lev,
                   [&](int32_t q) {
                     if (best.task_owner[q] != code) return false;
                     // updates of another node's tiles: the leader only
                     return all[q].kind == 0 || slot_own[all[q].dst] == code || F.leader;
                   },
                   F.ftask, F.flevel, F.fpanels);
      build_dataflow_deps(P, F.ftask, F.flevel, F.fdep_start, F.fdep);
      F.fqueue = queue_order(P, F.ftask, F.flevel, F.fdep_start, F.fdep, queue_workers());
      rhs_lists(code, F.rhs_tile, F.rhs_start, F.rhs_slot);
    }
    // backward: this rank's separator columns first (the top of the tree),
    // then its interior, in the global level order
    std::vector<int32_t> mine_codes;
    for (int32_t nd : path) mine_codes.push_back(sep_code(nd));
    std::vector<BackPart> keep;
    std::vector<int32_t> klev(1, 0);
    for (int pass = 0; pass < 2; ++pass) {
      for (size_t l = 0; l + 1 < P.bplevel.size(); ++l) {
        for (int32_t q = P.bplevel[l]; q < P.bplevel[l + 1]; ++q) {
          const int32_t o = P.tile_owner[P.bpart[q].k];
          const bool take = pass == 0 ? std::find(mine_codes.begin(), mine_codes.end(), o) != mine_codes.end()
                                      : o == P.rank;
          if (take) keep.push_back(P.bpart[q]);
        }
        if (static_cast<int32_t>(keep.size()) != klev.back()) klev.push_back(static_cast<int32_t>(keep.size()));
      }
    }
    P.bpart = std::move(keep);
    P.bplevel = std::move(klev);
  }
  bmark("rows, partition");
  build_dataflow_deps(P, P.ftask, P.flevel, P.fdep_start, P.fdep);
  bmark("dataflow deps");
  P.fqueue = queue_order(P, P.ftask, P.flevel, P.fdep_start, P.fdep, queue_workers());
  bmark("queue order");
  return true;
}

}  // namespace dynohip

extern "C" void dynohip_set_tile_ordering(int leaf) { dynohip::g_leaf_override = leaf < 0 ? -1 : leaf; }

extern "C" int dynohip_plan_schedule(const dynohip_graph_view* g, const uint64_t* keys, const uint8_t* kind, size_t n,
                                     dynohip_schedule_info* info, int32_t* tile_pos, int32_t* ftask,
                                     int32_t* pairs, int32_t* flevel, int32_t* btask, int32_t* blevel, int32_t* bent,
                                     int32_t* row_start, int32_t* row_col, int32_t* row_slot, int32_t* red_a,
                                     int32_t* red_b) {
  using namespace dynohip;
  if (!g || !info || (n && (!keys || !kind))) return DYNOHIP_EINVAL;
  Plan P;
  std::string err;
  const int rc = build_plan(*g, keys, kind, n, P, err);
  if (rc) return rc;
  info->n_pose = P.n_pose;
  info->n_tiles = P.NT;
  info->n_slots = P.n_slots;
  info->n_ftask = static_cast<int64_t>(P.ftask.size());
  info->n_pairs = static_cast<int64_t>(P.pairs.size() / 2);
  info->n_flevel = static_cast<int64_t>(P.flevel.size());
  info->n_btask = static_cast<int64_t>(P.btask.size());
  info->n_blevel = static_cast<int64_t>(P.blevel.size());
  info->n_bent = static_cast<int64_t>(P.bent.size() / 2);
  info->n_red_blocks = static_cast<int64_t>(P.red_A.size());
  info->nd_leaf = P.nd_leaf;
  auto put = [](int32_t* dst, const void* src, size_t bytes) {
    if (dst && bytes) std::memcpy(dst, src, bytes);
  };
  put(tile_pos, P.tile_pos.data(), P.tile_pos.size() * 4);
  put(ftask, P.ftask.data(), P.ftask.size() * sizeof(TileTask));
  put(pairs, P.pairs.data(), P.pairs.size() * 4);
  put(flevel, P.flevel.data(), P.flevel.size() * 4);
  put(btask, P.btask.data(), P.btask.size() * sizeof(BackTask));
  put(blevel, P.blevel.data(), P.blevel.size() * 4);
  put(bent, P.bent.data(), P.bent.size() * 4);
  put(row_start, P.row_start.data(), P.row_start.size() * 4);
  put(row_col, P.row_col.data(), P.row_col.size() * 4);
  put(row_slot, P.row_slot.data(), P.row_slot.size() * 4);
  put(red_a, P.red_A.data(), P.red_A.size() * 4);
  put(red_b, P.red_B.data(), P.red_B.size() * 4);
  return DYNOHIP_OK;
}
