// plan.hpp — host-side analysis of a factor graph into the device layout.
//
// Built once per dynohip_set_graph/set_values (the reference re-derives the
// equivalent structure on every solve: COLAMD + symbolic elimination inside
// GTSAM's NonlinearOptimizer::solve, called from RGBDBackendModule.cc:220,
// 374). Everything here is integer index work and is deterministic.
//
// Device layout (all FP64 data lives in one "arena"; gather lists address
// it with 32-bit double offsets):
//   factor records   per type, per factor: [J_slot0 | J_slot1 | ... | b]
//                    (each J block dim x slot_dim row-major, whitened and
//                    Huber-reweighted; b = -whitened residual)
//   D[n_pt]  (3x3)   point diagonal blocks      sum J_p^T J_p
//   E[n_pt]  (3x3)   chain sub-diagonal blocks  C_{i+1,i} = sum J_{i+1}^T J_i
//   gp[n_pt] (3)     point gradients            sum J_p^T b
//   W[n_edge](3x6)   point-pose coupling        sum J_p^T J_X
//   Y        (3x6)   C^-1 W per (component, point, neighbour pose)
//   v[n_pt]  (3)     C^-1 gp
//   L, M[n_pt](3x3)  block-Cholesky factors of each point chain
// Reduced (Schur) pose system: 64x64 tiles (tile t = reduced rows
// 64t..64t+63, poses in frame order: X_k, then H/L_{j,k}), stored sparsely
// by slot (see tiles.cpp) and factored by a level-scheduled tile DAG.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "../../include/dynohip.h"

namespace dynohip {

constexpr int kNTypes = 6;
constexpr int kNKeys[kNTypes] = {2, 3, 2, 1, 4, 3};
constexpr int kDim[kNTypes] = {3, 3, 6, 6, 3, 6};
constexpr int kMeasDim[kNTypes] = {3, 0, 12, 12, 0, 0};
constexpr int kCols[kNTypes] = {9, 12, 12, 6, 18, 18};
// 0 = pose slot, 1 = point slot, -1 unused
constexpr int kSlotKind[kNTypes][4] = {{0, 1, -1, -1}, {1, 1, 0, -1}, {0, 0, -1, -1},
                                       {0, -1, -1, -1}, {1, 1, 0, 0}, {0, 0, 0, -1}};
constexpr int kColStart[kNTypes][4] = {{0, 6, 0, 0}, {0, 3, 6, 0}, {0, 6, 0, 0},
                                       {0, 0, 0, 0}, {0, 3, 6, 12}, {0, 6, 12, 0}};
constexpr int kTile = 64;
constexpr int kRedBlock = 256;   // threads of a k_gather_reduced workgroup (kernels.hip kBlock)

// sum_e sign * A_e^T B_e, A_e: k x R, B_e: k x C (row-major blocks);
// sign kAddBlock: A_e is the R x R identity (a = Plan::off_I6), and the
// R x C block B_e is added as it is (the same bits as the identity product:
// every other row adds an exact zero), without the identity's row loads
constexpr int32_t kAddBlock = 2;
struct GEntry {
  uint32_t a;
  uint32_t b;
  int32_t k;
  int32_t sign;
};

// Lone-point group (k_lone_schur): up to lone_cap(m) lone points (static
// landmarks) sharing one sorted list of m neighbour poses, every point with
// exactly one PoseToPoint factor per neighbour and no other factor (a group
// of more points is split into several). Its workgroup sums the group's
// contributions to the reduced system into arena + out: the m(m+1)/2
// pose-pair blocks (a >= b, index a(a+1)/2 + b, 6x6 row-major, row = pose
// a) of H_cc - W_a^T D^-1 W_b, then the m 6-vector gradients
// J_a^T b - W_a^T D^-1 g_p. The reduced gathers read them as (identity,
// partial) entries. On the device a group is one block of kLoneBlk ints:
// [m, npt, out, 0, point[kLoneSub], first edge[kLoneSub],
//  neighbour pose[kLoneMaxNb], PoseToPoint record offset (J_pose at +0, b
//  at +27)[npt][m]].
// The group's arena area at `out` holds those per-try partials (36 m(m+1)/2
// + 6 m doubles), then its H area (42 m: the 6x6 J_a^T J_a per neighbour,
// then the J_a^T b), written once per linearisation by the fused
// linearisation (kernels.hip lone_lin_block).
// A block's kernels run a lane per (point, neighbour) in four 64-lane waves,
// floor(64 / m) points per wave: lone_cap(m) points (32 for the 7-pose
// tracks of the formulations' static landmarks).
constexpr int kLoneMaxNb = 10;
constexpr int kLoneSub = 32;
constexpr int kLoneHdrPt = 4;                             // point[kLoneSub]
constexpr int kLoneHdrE0 = kLoneHdrPt + kLoneSub;         // first edge[kLoneSub]
constexpr int kLoneHdrPose = kLoneHdrE0 + kLoneSub;       // neighbour pose[kLoneMaxNb]
constexpr int kLoneHdrRec = kLoneHdrPose + kLoneMaxNb;    // record offset[npt][m], npt m <= 256
constexpr int kLoneBlk = (kLoneHdrRec + 256 + 3) / 4 * 4;
constexpr int lone_cap(int m) { return 4 * (64 / m) < kLoneSub ? 4 * (64 / m) : kLoneSub; }
static_assert(lone_cap(1) * 1 <= 256 && lone_cap(kLoneMaxNb) * kLoneMaxNb <= 256, "a lane per (point, neighbour)");
struct LoneGroup {
  int32_t m;        // neighbour poses
  int32_t npt;      // member points
  int32_t pose_beg; // neighbour poses: lone_pose[pose_beg .. + m)
  uint32_t out;     // arena offset of the partial blocks
};

// one workgroup task of the tile Cholesky (see tiles.cpp / tilechol.hip).
// Operand pairs (A, B) index Plan::pairs; a pair stands for A B^T.
struct TileTask {
  int32_t kind;    // 0 = panel, 1 = update
  int32_t k;       // panel: column tile
  int32_t i;       // panel: row tile (== k for the diagonal task)
  int32_t dst;     // slot written: L(i,k) (panel) / updated tile (update)
  int32_t diag;    // panel: slot of A(k,k)
  int32_t pd_beg;  // panel: pending updates of A(k,k), pairs [pd_beg, pd_end)
  int32_t pd_end;
  int32_t po_beg;  // panel: pending updates of A(i,k) / update: its pairs
  int32_t po_end;
  int32_t pad;
};

// backward-substitution task: x_k = L_kk^-T (y_k - sum L(i,k)^T x_i)
struct BackTask {
  int32_t k;
  int32_t beg, end;  // entries [beg, end) of the (slot, row tile) list
  int32_t pad;
};

// one workgroup of a backward level: a slice [beg, end) of column k's
// entries; the nparts workgroups of a column meet through partial sums at
// partials + (pbase + part) * 64 and a per-column arrival counter
struct BackPart {
  int32_t k;
  int32_t beg, end;
  int32_t nparts, part, pbase;
  int32_t pad0, pad1;
};
// the one-launch backward solve keeps all its workgroups resident: at most
// this many (256 CUs x several 256-thread, few-KB-LDS workgroups each)
constexpr int kBackPersistMax = 1024;

// resize() leaves new elements uninitialised (large gather lists are filled
// completely right after; zeroing them first costs a pass of page faults)
template <typename T, typename A = std::allocator<T>>
struct default_init_allocator : A {
  using A::A;
  template <typename U>
  struct rebind {
    using other = default_init_allocator<U, typename std::allocator_traits<A>::template rebind_alloc<U>>;
  };
  template <typename U>
  void construct(U* p) noexcept(std::is_nothrow_default_constructible<U>::value) {
    ::new (static_cast<void*>(p)) U;
  }
  template <typename U, typename... Args>
  void construct(U* p, Args&&... args) {
    std::allocator_traits<A>::construct(static_cast<A&>(*this), p, std::forward<Args>(args)...);
  }
};

struct GatherList {
  std::vector<int64_t> start;  // ntargets + 1
  std::vector<GEntry, default_init_allocator<GEntry>> ent;
  size_t ntargets() const { return start.empty() ? 0 : start.size() - 1; }
};

struct TypePlan {
  int n = 0;
  uint64_t base = 0;     // arena offset of the first record
  uint32_t stride = 0;   // doubles per record
  std::vector<int32_t> idx;   // n * nkeys (pose index or point index per slot)
  std::vector<double, default_init_allocator<double>> meas;    // n * meas_dim
  std::vector<double, default_init_allocator<double>> isig;    // n * dim (1/sigma)
  std::vector<double, default_init_allocator<double>> hk;      // n (Huber k, <= 0 Gaussian)
};

// Partitioned solve: a separator of the top dissection levels (tiles.cpp
// nd_order_part). The ranks [r0, r0 + nr) of the subtree it splits factor it
// after the exchange of its depth (1: the top separator); r0 leads the group
// (it alone passes the node's contributions on to the separators above).
// Tiles [t0, t1) in natural order.
struct SepNode {
  int32_t r0, nr, depth, t0, t1;
};
// tile / task owner of a separator node's columns (ranks are >= 0)
constexpr int32_t sep_code(int32_t node) { return -1 - node; }
constexpr int32_t sep_node(int32_t code) { return -1 - code; }

// One phase of a rank's partitioned solve after its interior (phase 0): the
// exchange of one depth's separator systems, then the tasks of this rank's
// separator node of that depth.
struct PartPhase {
  int32_t node = 0;                     // the node whose columns this phase factors
  int32_t leader = 0;                   // 1: this rank leads the node's group
  // summed over all ranks before the phase: [beg, end) slot ranges of every
  // node of this depth, and their right-hand-side tile ranges (natural order)
  std::vector<int32_t> xslot, xtile;
  std::vector<TileTask> ftask;          // the node's tasks on this rank (dataflow form as Plan::ftask)
  std::vector<int32_t> flevel, fpanels, fdep_start, fdep, fqueue;
  // after the phase: the node's column contributions L(s,c) y_c to rows s of
  // separators above it leave the RHS (leader: r_s -= them; every member:
  // the contribution is cleared), k_sep_rhs's lists
  std::vector<int32_t> rhs_tile, rhs_start, rhs_slot;
};

struct Plan {
  // variables
  int n_pose = 0, n_pt = 0;
  std::vector<uint8_t> user_kind;   // per user value
  std::vector<int32_t> user_idx;    // pose index or point index
  std::vector<uint64_t> pose_key, pt_key;
  // point components (chains), points contiguous in chain order
  int n_comp = 0;
  int max_chain = 0;
  std::vector<int32_t> comp_start;      // n_comp + 1
  std::vector<int32_t> comp_nb_start;   // n_comp + 1 (into nb arrays)
  std::vector<int32_t> nb_pose;         // per nb entry
  std::vector<int32_t> nb_comp;         // per nb entry
  std::vector<int64_t> comp_y_base;     // arena offset of comp's Y
  std::vector<int32_t> nbedge_start;    // per nb entry + 1
  std::vector<int32_t> nbedge_pt;       // local point index in comp
  std::vector<uint32_t> nbedge_w;       // arena offset of W block
  // point-pose edges, sorted by (point, pose)
  int n_edge = 0;
  std::vector<int32_t> edge_pt, edge_pose;
  std::vector<int32_t> pt_edge_start;   // n_pt + 1
  TypePlan types[kNTypes];
  // gathers
  GatherList gD, gE, gGp, gW, gRed, gGred;
  std::vector<int32_t> red_A, red_B;    // reduced target pose indices (A >= B)
  // per target, the slots of the (up to) 2 x 2 tiles its 6x6 block touches:
  // [row tile of 6A / of 6A+5][col tile of 6B / of 6B+5], bit 31 = the tile is
  // stored transposed (its column tile is eliminated later); ~0u: not stored
  std::vector<uint32_t> red_slot;
  // the targets by entry count, for k_gather_reduced's lane groups: targets
  // of <= 4, <= 8, <= 16, <= 32 and more entries (kRedClasses), each class in
  // target order; red_ncls = targets per class
  static constexpr int kRedClasses = 5;
  std::vector<int32_t> red_order;
  int32_t red_ncls[kRedClasses] = {};
  // k_gather_reduced's band blocks in column order: entry (k << 3) | c is
  // block k of class c (its targets red_order[class offset + k * per-block
  // targets ...]), blocks sorted by the column (red_B) of their first
  // target, so every class's targets of a column band run at the same time
  // and on the same XCD (plan.cpp compute_red_slots)
  std::vector<int32_t> red_blocks;
  // lone-point groups (k_lone_schur); their points' factor pairs and
  // component pairs are not in gRed / gGred
  std::vector<LoneGroup> lgroup;
  std::vector<int32_t> lone_pose;
  std::vector<int32_t, default_init_allocator<int32_t>> lone_blk;   // kLoneBlk per group (device form)
  int lone_max_m = 0;
  bool lone_all_grouped = false;        // every lone point is in a group (no lone Y is read)
  // the PoseToPoint factors outside the lone groups, in factor order: the
  // ones k_linearize still records when the groups linearise their own
  // factors (k_lone_lin, the fused static landmarks)
  std::vector<int32_t> lin_list0;
  uint64_t off_I6 = 0;                  // 6x6 identity (the A operand of the partial entries)
  // arena
  uint64_t off_D = 0, off_E = 0, off_gp = 0, off_W = 0, off_Y = 0, off_v = 0, off_L = 0, off_M = 0;
  uint64_t arena_size = 0;
  // reduced system
  int n_red = 0;                        // 6 * n_pose
  int NT = 0;                           // tiles
  std::vector<int32_t> band_D;          // natural-order skyline: sub-diagonal tiles per column tile
  int max_D = 0;
  // tile Cholesky (tiles.cpp)
  int nd_leaf = 0;                      // chosen nested-dissection leaf size (0 = natural order)
  std::vector<int32_t> tile_pos;        // elimination position of tile t
  int32_t n_slots = 0;                  // stored tiles (lower factor incl. fill)
  std::vector<int32_t> row_start;       // per tile t: stored tiles whose row tile is t
  std::vector<int32_t> row_col;         //   their column tiles (sorted)
  std::vector<int32_t> row_slot;        //   and slots
  std::vector<TileTask> ftask;          // forward tasks, grouped by level
  std::vector<int32_t> pairs;           // operand pairs (A slot, B slot) of the tasks
  std::vector<int32_t> flevel;          // level l = tasks [flevel[l], flevel[l+1])
  std::vector<int32_t> fpanels;         // panels of level l (they come first within the level)
  // dataflow form of the same schedule (k_factor_persist): task q may start
  // once every slot of fdep[fdep_start[q] .. fdep_start[q+1]) (pairs: slot,
  // count) has received `count` completed writes (update tasks and panels
  // i != k write their dst slot once each)
  std::vector<int32_t> fdep_start;
  std::vector<int32_t> fdep;
  // the dataflow kernel's queue: task ids in the order the workgroups take
  // them, a list schedule of the dependency graph (tiles.cpp queue_order)
  std::vector<int32_t> fqueue;
  std::vector<BackTask> btask;
  std::vector<int32_t> blevel;
  std::vector<int32_t> bent;            // pairs (slot, row tile)
  int32_t back_part_tiles = 2;          // entries (64x64 tiles) per backward workgroup
  std::vector<BackPart> bpart;          // backward workgroups, grouped by level
  std::vector<int32_t> bplevel;         // level l = bpart [bplevel[l], bplevel[l+1])
  int32_t n_partials = 0;
  double tile_flops = 0.0;              // tile-level factorisation flops (incl. fill)
  // partitioned full-batch solve. nranks > 1: the
  // lists above hold this rank's phase-0 tasks (its interior) and its
  // backward parts (its separator nodes' columns first, then its interior);
  // `phases` the separator phases, deepest node first, the top one last
  int nranks = 1, rank = 0;
  std::vector<int32_t> tile_owner;      // per tile: owning rank, or sep_code(node)
  std::vector<SepNode> sep_nodes;
  std::vector<PartPhase> phases;
  // phase 0's right-hand-side move (k_sep_rhs): this rank's interior column
  // contributions to separator rows
  std::vector<int32_t> rhs0_tile, rhs0_start, rhs0_slot;
  // build_plan's largest temporaries, kept with the plan (not plan content):
  // a re-plan of a similar graph refills memory that is already mapped
  // instead of page-faulting fresh allocations (C2 ~7 MB, NS ~25 MB)
  struct Scratch {
    std::vector<uint64_t> key_k;
    std::vector<int32_t> key_v;
    std::vector<int32_t, default_init_allocator<int32_t>> fuser[kNTypes];
    std::vector<int32_t> adj, cnt;
    std::vector<int32_t, default_init_allocator<int32_t>> poses;
    std::vector<int64_t> rstart;
    std::vector<uint64_t, default_init_allocator<uint64_t>> refs;
    std::vector<uint32_t> prec;
  } scratch;
};

// Resets `P` to a default Plan but keeps the capacity of its arrays: the
// next build_plan of a similar graph refills memory that is already mapped
// and touched instead of faulting fresh pages in (and freeing the old ones).
void plan_recycle(Plan& P);

// Orders the tiles (nested dissection over frame order), computes the
// tile-level fill and the task DAG with its level schedule. With
// P.nranks > 1 the top of the dissection is split into rank subtrees; false
// when the graph is too short for that many.
// own_threads: the candidate orderings run on threads of their own instead
// of the planner pool (the schedule then runs beside the gather builds).
bool build_tile_schedule(Plan& P, bool own_threads = false);

// The tile owners of the partitioned schedule (per natural tile: rank, or
// sep_code(node)) and the separator nodes, from the pose-pair structure
// alone: the top splits of the dissection do not depend on the leaf size, so
// this equals the schedule's tile_owner. False when the graph is too short in
// time for nranks.
bool partition_tile_owners(const Plan& P, int nranks, std::vector<int32_t>& owner, std::vector<SepNode>& nodes);

// Plan::red_slot from the tile structure (after the tile schedule).
void compute_red_slots(Plan& P);

// returns DYNOHIP_OK or an error code with `err` filled. nranks > 1 builds
// the partitioned tile schedule of `rank` (the graph is the global one);
// with_schedule = false stops after the reduced-system structure.
// structure_only = true builds no gather lists and no lone-point groups:
// the point chains, the reduced system's pose-pair blocks and (with
// with_schedule) the tile schedule only, which is all the partitioned plan
// needs of the global graph.
// Called by build_plan as parts of the plan become final (the caller may
// start uploading them while the planner goes on).
struct PlanHook {
  virtual ~PlanHook() = default;
  // P.types (indices, measurements, 1/sigma, Huber k) are final
  virtual void types_ready(const Plan& P) = 0;
};

int build_plan(const dynohip_graph_view& g, const uint64_t* keys, const uint8_t* kind, size_t n, Plan& plan,
               std::string& err, int nranks = 1, int rank = 0, bool with_schedule = true, bool structure_only = false,
               PlanHook* hook = nullptr);

// Partitioned full-batch solve: what one rank holds (partition.cpp).
struct Partition {
  int nranks = 1, rank = 0;
  std::vector<int32_t> value_owner;     // per global value: owning rank (a separator pose: its node's leader, nodes[].r0)
  std::vector<int32_t> local_of;        // per global value: index in the local value list, -1 = not held
  std::vector<uint64_t> keys;           // local value list (all poses + this rank's points)
  std::vector<uint8_t> kind;
  std::vector<int32_t> global_of;       // per local value: global index
  std::vector<uint8_t> damp_row;        // per reduced row: this rank adds lambda
  size_t factors_local = 0, factors_total = 0;
};

// Splits the global graph over nranks time-contiguous subtrees of the
// nested dissection; builds this rank's local plan (its factors, all poses,
// its points) carrying the global partitioned tile schedule. `local_graph`
// receives the storage the local plan's graph view points into.
struct GraphStore {
  std::vector<uint64_t> keys[kNTypes];
  std::vector<double> meas[kNTypes], sig[kNTypes], hub[kNTypes];
  size_t n[kNTypes] = {};
  dynohip_graph_view view() const;
};
int build_partitioned_plan(const dynohip_graph_view& g, const uint64_t* keys, const uint8_t* kind, size_t n,
                           int nranks, int rank, Plan& local, Partition& part, GraphStore& local_graph,
                           std::string& err);

}  // namespace dynohip
