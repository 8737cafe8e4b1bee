// kernels.hpp — device data views and launchers for the HIP hot path.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "plan.hpp"

namespace dynohip {

struct TypeDev {
  int n = 0;
  uint64_t base = 0;
  uint32_t stride = 0;
  const int32_t* idx = nullptr;
  const double* meas = nullptr;
  const double* isig = nullptr;
  const double* hk = nullptr;
  // k_linearize only: the factors to linearise are list[0, n) (factor ids),
  // null = factors 0 .. n-1 (the fused static landmarks leave theirs out)
  const int32_t* list = nullptr;
};

struct GatherDev {
  int n = 0;
  const int64_t* start = nullptr;
  const GEntry* ent = nullptr;
};

// launch_gather_point: D, E, g_p, W targets
struct PointGatherDev {
  GatherDev g[4];
  double* dst[4] = {};
  int bstart[5] = {};
  // lone-point groups (plan.hpp LoneGroup): a workgroup per group block
  // forms D, g_p and W of its points from their PoseToPoint records
  int n_lone = 0;
  const int32_t* lone_blk = nullptr;
};

struct ReducedGatherDev {
  GatherDev band;              // 6x6 reduced blocks (targets tA[t], tB[t])
  // the targets by entry count (Plan::red_order): class c, of <= 4 << c
  // entries, runs 8 << c lanes per target (two per entry; the last class
  // 128 lanes), its targets at order[ooff[c], + ncls[c]); dispatch position d
  // (blocks [bstart[d], bstart[d+1])) runs class cls[d]
  static constexpr int kClasses = 5;
  const int32_t* order = nullptr;
  int ncls[kClasses] = {};
  int ooff[kClasses] = {};
  int cls[kClasses] = {};
  int bstart[kClasses + 1] = {};
  const int32_t* tA = nullptr;
  const int32_t* tB = nullptr;
  const uint32_t* tslot = nullptr;   // Plan::red_slot
  GatherDev grad;              // 6-vector reduced gradient per pose
  double* gred = nullptr;
  int nb_band = 0, nb_grad = 0;
  const uint8_t* damp = nullptr;  // partitioned: per reduced row, 1 = this rank adds lambda (null: every row)
  // Plan::red_blocks (null: each class's blocks in turn, bstart/cls)
  const int32_t* blocks = nullptr;
};

// buffers zeroed by the blocks past the chains in k_chain_factor, and
// buffers filled with kBackSentinel (k_back_poll's x and partials)
struct ZeroDev {
  double* p[3] = {};
  int64_t n[3] = {};           // doubles, even
  double* s[2] = {};
  int64_t sn[2] = {};          // doubles, even
};

struct ChainDev {
  int n_comp = 0;
  int n_nb = 0;
  int n_long = 0;      // chains of >= 2 points: comps [0, n_long) (longest first)
  int n_nb_long = 0;   // their (chain, neighbour pose) pairs: [0, n_nb_long)
  const int32_t* comp_start = nullptr;
  const int32_t* comp_nb_start = nullptr;
  const int32_t* nb_comp = nullptr;
  const int64_t* comp_y_base = nullptr;
  const int32_t* nbedge_start = nullptr;
  const int32_t* nbedge_pt = nullptr;
  const uint32_t* nbedge_w = nullptr;
  const int32_t* pt_edge_start = nullptr;
  const int32_t* edge_pose = nullptr;
  const int32_t* edge_pt = nullptr;
  int e_lone0 = 0;        // first edge of the lone points
  int n_lone_edges = 0;   // their edges (the Y blocks follow edge order from y_lone_base)
  uint64_t y_lone_base = 0;
  uint64_t off_D = 0, off_E = 0, off_gp = 0, off_W = 0, off_v = 0, off_L = 0, off_M = 0;
};

// lone-point groups (plan.hpp LoneGroup), a workgroup per group
struct LoneSchurDev {
  int n_group = 0;
  int max_m = 0;                          // largest m (sizes the staging LDS)
  const int32_t* blk = nullptr;           // kLoneBlk ints per group
  uint64_t off_W = 0, off_L = 0, off_gp = 0, off_I6 = 0;
  uint64_t off_D = 0, off_v = 0;          // (launch_chain_lone: the groups factor their points)
  // fused: J_a^T J_a and J_a^T b come from the group's H area (the fused
  // linearisation, plan.hpp), not from the PoseToPoint records
  int fused = 0;
};

// fused static-landmark linearisation (k_lone_lin), a workgroup per lone
// group block: evaluates the block's PoseToPoint factors and writes W (per
// edge), D and g_p (per point), the block's per-pose sums J_a^T J_a, J_a^T b
// (its H area) and its share of the linear error at delta = 0
struct LoneLinDev {
  int n_group = 0;
  const int32_t* blk = nullptr;
  TypeDev t0;                             // PoseToPoint factor data (record offset -> factor id via base, stride)
  uint64_t off_W = 0, off_D = 0, off_gp = 0;
};

// reduced system in 64x64 tiles; tile (row tile i, column tile j) with
// pos[i] >= pos[j] lives at slots + slot * 4096 (row-major)
struct TileDev {
  int NT = 0;
  int n_red = 0;
  double* slots = nullptr;
  const int32_t* pos = nullptr;
  const int32_t* row_start = nullptr;
  const int32_t* row_col = nullptr;
  const int32_t* row_slot = nullptr;
};

struct TileSchedDev {
  const TileTask* ftask = nullptr;
  const int32_t* pairs = nullptr;
  const BackPart* bpart = nullptr;
  const int32_t* bent = nullptr;
  double* partials = nullptr;  // n_partials x 64
  int* arrive = nullptr;       // NT arrival counters (zero between launches)
  unsigned* done = nullptr;    // NT column-done stamps of the one-launch backward solve
  unsigned epoch = 0;          // stamp of the current solve (never 0)
  const int32_t* fdep_start = nullptr;  // dataflow dependencies (Plan::fdep)
  const int32_t* fdep = nullptr;
  const int32_t* forder = nullptr;  // the dataflow queue: task ids in the order workgroups take them
  unsigned* wcnt = nullptr;    // per-slot write counters, zeroed before each solve
  unsigned* fqueue = nullptr;  // task queue head, zeroed before each solve
  bool persistent_factor = true;  // one dataflow launch instead of one launch per level
  int workers = 256;           // its workgroups (one per CU)
  int wide_updates = 256;      // levels with more update tasks use the side-stream kernel
  bool level_backward = false; // force one backward launch per level
  // one-launch backward: hand-offs on the data (k_back_poll; x and partials
  // sentinel-filled before each solve) instead of epoch flags (k_back_persist)
  bool back_poll = true;
};

// the sentinel k_back_poll's consumers wait past (a signalling NaN)
constexpr uint64_t kBackSentinel = 0xFFF4DEADBEEFCAFEull;

// ---- launchers (all asynchronous on `s`) ----
// Factor kernels, one launch per type group. Partials are laid out in type
// order (error_blocks slots). With out != nullptr the last launch also sums
// all partials into *out (counter: a zeroed device word, left zeroed);
// launch_linearize's sum is the linear error at delta = 0.
int error_blocks(const TypeDev* td);
// lone (optional): the fused static landmarks' group blocks (W, D, g_p of
// the grouped lone points, the groups' H areas) run as the first workgroups
// of the PoseToPoint launch, their linear error joining the sum. Returns -1
// without launching when lone's tables are null.
int linearize_blocks(const TypeDev* td, const LoneLinDev* lone = nullptr);
int launch_linearize(const TypeDev* td, const double* pose, const double* pt, double* arena, double* partials,
                     unsigned* counter, double* out, hipStream_t s, const LoneLinDev* lone = nullptr);
// fail_src (optional): accumulated failure bits, moved to *fail_dst and cleared
// extra_* (optional): the finishing block also sums extra_in[0, extra_n) in
// order into *extra_out (the back-substitution's cost-change partials)
void launch_error(const TypeDev* td, const double* pose, const double* pt, double* partials, unsigned* counter,
                  double* out, int* fail_src, int* fail_dst, hipStream_t s, const double* extra_in = nullptr,
                  int extra_n = 0, double* extra_out = nullptr);
void launch_linerr(const TypeDev* td, const double* arena, const double* dpose, const double* dpt, double* partials,
                   unsigned* counter, double* out, hipStream_t s);

// point-side gathers (thread per target), dst = arena + off
void launch_gather_point(const GatherDev (&g)[4], double* const (&dst)[4], const double* arena, hipStream_t s,
                         int n_lone = 0, const int32_t* lone_blk = nullptr);
// reduced blocks into their tiles (+ lambda), reduced gradient, identity padding
void launch_gather_reduced(const GatherDev& band, const int32_t* order, const int32_t* ncls, const int32_t* tA, const int32_t* tB, const uint32_t* tslot,
                           const GatherDev& grad,
                           double* gred, const double* arena, const TileDev& b, double lambda, hipStream_t s,
                           const uint8_t* damp = nullptr, const int32_t* blocks = nullptr, int n_blocks = 0);
// partitioned: r[rows of separator tile] -= sum of this rank's contributions
// L(s,c) y_c (c interior), which are then zeroed; CSR over separator tiles
// Plan upload: one host-to-device copy of a staged block, then this kernel
// places its pieces (chunks of <= 64 KB, 16-byte aligned) into their device
// arrays.
struct CopyChunk {
  uint64_t dst;      // device address
  uint32_t src_off;  // from the staged data's start, in 256-byte units
  uint32_t bytes;
};
void launch_scatter_chunks(const char* data, const CopyChunk* chunks, int n_chunks, hipStream_t s);

void launch_sep_rhs(int n_sep_tiles, const int32_t* tile, const int32_t* start, const int32_t* slot, double* r,
                    double* contrib, int apply, hipStream_t s);

void launch_chain_factor(const ChainDev& c, double* arena, double lambda, int* fail, const ZeroDev& z,
                         hipStream_t s);
void launch_chain_solve_y(const ChainDev& c, double* arena, hipStream_t s);
// the lone-point groups' partial reduced blocks and gradients (after
// launch_chain_factor: reads L and v of the lone points)
void launch_lone_schur(const LoneSchurDev& d, double* arena, hipStream_t s);
// every lone point grouped: the groups (with their points' factorisation,
// L and v) and k_chain_factor's long chains and fill blocks in one launch,
// in place of launch_chain_factor + launch_lone_schur
void launch_chain_lone(const ChainDev& c, const LoneSchurDev& d, double* arena, double lambda, int* fail,
                       const ZeroDev& z, hipStream_t s);
int debug_lone_clock(void* out);   // -DDYNOHIP_LONE_CLOCK builds: the stamps of the last launch
// The tail of a try in the back-substitution launch (LevenbergMarquardt-
// Optimizer.cpp tryLambda): the candidate values and the linearised cost
// change, formed from the solve itself instead of re-reading the Jacobian
// records (JacobianFactor::error over the graph). With (H + lambda I) delta
// = g (GTSAM's default damping, lambda on every dimension) and
// L(delta) = 0.5 ||J delta - b||^2:
//   L(0) - L(delta) = 0.5 (delta^T g + lambda ||delta||^2),
//   delta^T g = dx^T g_red + sum over points (t^T v + dp^T g_p),
// t = W dx, v = C^-1 g_p (k_chain_factor), g_red the reduced gradient
// (g_x = g_red + W^T v). Each block of the launch leaves its partial of
// delta^T g + lambda ||delta||^2 in `partials` (launch_error's finishing block
// sums them in block order); the point lanes write pt_out = pt + dp and the
// pose blocks (a thread per pose) pose_out = pose * Exp(dx), so no separate
// retraction launch runs.
struct LinChangeDev {
  double* partials = nullptr;   // one slot per block of the launch (backsub_blocks)
  double* out = nullptr;        // non-null: this tail runs (the sum lands here)
  const double* gred = nullptr;
  int n_pose = 0;               // x in pose order, 6 per pose
  double lambda = 0.0;
  const double* pose = nullptr;
  const double* pt = nullptr;
  double* pose_out = nullptr;
  double* pt_out = nullptr;
};
// blocks of the back-substitution launch (the partial slots LinChangeDev needs)
int backsub_blocks(const ChainDev& c, int n_lone, int n_pose);
// dpt = C^-1 (gp - W dpose);
// lc (optional): the linearised cost change as above
void launch_backsub(const ChainDev& c, const double* arena, const double* dpose, double* dpt,
                    hipStream_t s, int n_lone = 0, const int32_t* lone_blk = nullptr,
                    const LinChangeDev* lc = nullptr);

// factor the tiles and solve (L L^T) x = r (forward substitution fused
// into the factorisation: contrib holds L(i,k) y_k per stored tile). Linv
// receives the NT diagonal inverse tiles, y the forward result. One launch
// per level of the host schedule (flevel / bplevel).
// Wide levels (many update tasks) run their updates as a separate
// small-LDS kernel on `side`, concurrently with the level's panels on `s`
// (joined through ev_main / ev_side).
// (launch_tile_backward after it completes the solve; the partitioned solve
// runs the forward tasks in two phases around the exchange)
void launch_tile_forward(const TileDev& b, const TileSchedDev& sd, const std::vector<int32_t>& flevel,
                         const std::vector<int32_t>& fpanels, double* Linv, const double* r, double* contrib,
                         double* y, int* fail, hipStream_t s, hipStream_t side, hipEvent_t ev_main,
                         hipEvent_t ev_side);
// the whole reduced solve of a system of <= kSmallNT tiles in one workgroup
// (x = A^-1 r in natural tile order; tilechol.hip k_small_solve)
constexpr int kSmallNT = 4;
// the small solve's view of the tiles: the tile at each elimination position
// and the slot of position block (p, q), p <= q (-1: no stored tile); filled
// on the host from the plan, so the kernel starts with no index round trips
struct SmallMap {
  int32_t ord[kSmallNT];
  int32_t slot[kSmallNT][kSmallNT];
};
void launch_small_solve(const TileDev& b, const SmallMap& m, const double* r, double* x, int* fail, hipStream_t s);
// sentinel_filled: x and sd.partials hold kBackSentinel for this solve (the
// hand-off form k_back_poll needs it; without it the flag form runs)
void launch_tile_backward(const TileDev& b, const TileSchedDev& sd, const std::vector<int32_t>& blevel,
                          const double* Linv, const double* y, double* x, int* fail, hipStream_t s,
                          bool sentinel_filled);

void launch_retract(int n_pose, int n_pt, const double* pose, const double* pt, const double* dpose,
                    const double* dpt, double* pose_out, double* pt_out, hipStream_t s);

}  // namespace dynohip
