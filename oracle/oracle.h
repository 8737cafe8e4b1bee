/*
 * oracle.h — CPU restatement of the DynoSAM backend hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker for the
 * HIP product path (dynosam_amd/csrc). Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it; the product never does.
 *
 * What it restates (reference file:line in /root/reference):
 *  - factors: gtsam::PoseToPointFactor (BackendDefinitions.hpp:54, GTSAM
 *    4.2.0 gtsam_unstable/slam/PoseToPointFactor.h), LandmarkMotionTernary
 *    (LandmarkMotionTernaryFactor.cc:37-73), BetweenFactor<Pose3>
 *    (FactorGraphTools.cc:73-83; GTSAM 4.2.0 BetweenFactor.h, default build
 *    i.e. GTSAM_SLOW_BUT_CORRECT_BETWEENFACTOR off, docker/Dockerfile:88),
 *    PriorFactor<Pose3> (Formulation-impl.hpp:91-104; GTSAM 4.2.0
 *    PriorFactor.h), LandmarkMotionPose (LandmarkMotionPoseFactor.cc:32-88),
 *    LandmarkPoseSmoothing (LandmarkPoseSmoothingFactor.cc:29-83) with
 *    gtsam::numericalDerivative (central, delta 1e-5);
 *  - noise: Isotropic/Diagonal whitening and Robust(Huber, Block)
 *    (BackendModule.cc:56-85, RGBDBackendModule.cc:89-117);
 *  - Pose3/Rot3 with GTSAM_POSE3_EXPMAP / GTSAM_ROT3_EXPMAP (Dockerfile:88);
 *  - gtsam::LevenbergMarquardtOptimizer 4.2.0 defaults, called at
 *    RGBDBackendModule.cc:207-221,364-376;
 *  - keys (BackendDefinitions.hpp:57-88, DynamicPointSymbol.cc:31-44).
 *
 * The damped normal equations are solved exactly, either by a dense
 * Cholesky of the full system (small graphs) or by Schur elimination of
 * point components followed by an envelope (skyline) Cholesky of the
 * frame-ordered reduced pose system.
 */
#ifndef DYNOHIP_ORACLE_H_
#define DYNOHIP_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#include "../include/dynohip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_problem oracle_problem;

int oracle_create(const dynohip_graph_view* g, const uint64_t* keys,
                  const uint8_t* kind, const double* data, size_t n,
                  oracle_problem** out);
void oracle_destroy(oracle_problem* p);
const char* oracle_last_error(const oracle_problem* p);
/* 0 = Schur + skyline (default), 1 = dense full-system Cholesky */
void oracle_set_dense(oracle_problem* p, int dense);
/* rounding control: the Schur solve sums factors and point components in
   reverse order (serial solve); the same mathematics, other rounding */
void oracle_set_reverse_sums(oracle_problem* p, int reverse);
/* every LM solve in x87 extended precision (test reference, serial) */
void oracle_set_solve_ld(oracle_problem* p, int on);
/* threads of the Schur + skyline LM (default 1); the trajectory is
   bit-identical for every thread count (the all-cores CPU baseline) */
int oracle_set_threads(oracle_problem* p, int nthreads);

double oracle_error(oracle_problem* p);
int oracle_lm_reset(oracle_problem* p, const dynohip_lm_params* prm);
int oracle_iterate(oracle_problem* p, dynohip_lm_summary* s);
int oracle_optimize(oracle_problem* p, const dynohip_lm_params* prm,
                    dynohip_lm_summary* s);
int oracle_get_values(const oracle_problem* p, double* out, size_t n_doubles);
int oracle_set_values_data(oracle_problem* p, const double* data,
                           size_t n_doubles);
int oracle_get_trace(const oracle_problem* p, dynohip_trace_entry* out,
                     size_t cap, size_t* n_out);
size_t oracle_linearize_size(const oracle_problem* p);
int oracle_linearize(oracle_problem* p, double* out, size_t n_doubles);
/* solve the damped system at the current linearisation point with a given
   lambda; delta is written in value order (6 per pose, 3 per point).
   returns 1 if solved, 0 if indefinite, <0 on error */
int oracle_solve_damped(oracle_problem* p, double lambda, double* delta_out,
                        size_t n_doubles);
/* the same step with the Schur solve in x87 extended precision (a reference
   for ill-conditioned deep-convergence systems); 1 = solved */
int oracle_solve_damped_ld(oracle_problem* p, double lambda, double* delta_out, size_t n_doubles);

/* factor-level hooks: type as in dynohip_graph_view order (0..5).
   vars: the factor's variable values in key order (12 per pose, 3 per
   point) concatenated; meas may be NULL. r: dim; J: dim x cols row-major
   (unwhitened). */
int oracle_eval_factor(int type, const double* vars, const double* meas,
                       double* r, double* J);
int oracle_factor_dim(int type);
int oracle_factor_cols(int type);
int oracle_factor_nkeys(int type);

/* Pose3 / Rot3 hooks (12-double poses) */
void oracle_pose_expmap(const double xi[6], double T[12]);
void oracle_pose_logmap(const double T[12], double xi[6]);
void oracle_pose_compose(const double A[12], const double B[12], double C[12]);
void oracle_pose_inverse(const double A[12], double C[12]);
void oracle_rot_expmap(const double w[3], double R[9]);
void oracle_rot_logmap(const double R[9], double w[3]);
/* the shared sin / tan / acos of trig.h: which 0, 1, 2 */
void oracle_trig(int which, const double* x, double* y, size_t n);

/* keys */
uint64_t oracle_cantor_pair(uint64_t k1, uint64_t k2);
void oracle_cantor_depair(uint64_t z, uint64_t* k1, uint64_t* k2);
uint64_t oracle_symbol(unsigned char c, uint64_t j);
uint64_t oracle_labeled_symbol(unsigned char c, unsigned char label,
                               uint64_t j);
int oracle_reconstruct_labeled(uint64_t key, unsigned char expected_chr,
                               int* label, uint64_t* frame);
unsigned char oracle_chr_extract(uint64_t key);

#ifdef __cplusplus
}
#endif

#endif
