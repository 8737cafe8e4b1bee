/*
 * dynorefine.h — batched object-motion refinement on the GPU (SURVEY.md
 * §8(f) row 4).
 *
 * Replaces, for a whole batch of (object, frame pair) problems at once,
 *   MotionOnlyRefinementOptimizer::optimize<Cal3_S2>(frame_k_1, frame_k,
 *       tracklets, object_id, initial_motion, ProjectionError)
 * (dynosam/include/dynosam/frontend/vision/MotionSolver-inl.hpp:277-470,
 *  called from ObjectMotionSovler, dynosam/src/frontend/vision/
 *  MotionSolver.cc:514-522). Per problem the graph is the reference's: priors
 * (sigma 1e-5) on X_{k-1} and X_k, per tracklet two
 * GenericProjectionFactor<Pose3, Point3, Cal3_S2> (Huber on Isotropic(2,
 * projection_sigma), throwCheirality = false) and one
 * LandmarkMotionTernaryFactor (Huber on Isotropic(3, landmark_motion_sigma)),
 * solved with gtsam::LevenbergMarquardtOptimizer default semantics, then
 * factor_graph_tools::determineFactorOutliers<LandmarkMotionTernaryFactor>
 * (FactorGraphTools.hpp:70-98, chi2(3, 0.99)).
 *
 * Outlier handling (MotionSolver-inl.hpp:405-437): with outlier_reject = 1
 * (the reference default) and at least one outlier, the reference inserts
 * the motion key into `values` a second time, which throws
 * gtsam::ValuesKeyAlreadyExists; the result then carries status
 * DYNOREFINE_VALUES_KEY_EXISTS (the detected outliers are flagged). 0 skips
 * the outlier step; 2 runs the loop the code intends (drop the outlier
 * ternary factors, re-solve from the optimised values, at most 4 rounds) —
 * a documented deviation, not the default.
 *
 * Plain C, host pointers; a handle owns its device buffers and is used from
 * one thread.
 *
 * Versioning: the layout of dynorefine_batch is covered by
 * DYNOHIP_ABI_VERSION (dynohip.h). Version 2 appended `ternary_inactive`; a
 * consumer checks dynohip_abi_version() == DYNOHIP_ABI_VERSION before
 * calling dynorefine_upload, since a batch built against an older header is
 * shorter and its missing trailing pointer would be read as garbage.
 */
#ifndef DYNOREFINE_H_
#define DYNOREFINE_H_

#include <stddef.h>
#include <stdint.h>

#include "dynohip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  size_t n_problems;
  const int32_t* track_start;  /* n_problems + 1: tracklets of problem p are
                                  [track_start[p], track_start[p+1])        */
  const double* X_k_1;         /* 12 per problem: frame_k_1->getPose()       */
  const double* X_k;           /* 12 per problem: frame_k->getPose()         */
  const double* H_init;        /* 12 per problem: initial_motion             */
  const double* calibration;   /* 5 per problem: Cal3_S2 fx, fy, s, u0, v0   */
  const double* kp_k_1;        /* 2 per tracklet: keypoint at k-1            */
  const double* kp_k;          /* 2 per tracklet: keypoint at k              */
  const double* m_k_1;         /* 3 per tracklet: backProjectToWorld at k-1  */
  const double* m_k;           /* 3 per tracklet: backProjectToWorld at k    */
  /* Optional initial values of X_{k-1}, X_k (12 per problem) when they
     differ from the prior measurements X_k_1 / X_k (null: the same, as in
     the reference). Lets a test restart the solver from any LM state. */
  const double* X_k_1_init;
  const double* X_k_init;
  /* Optional, 1 per tracklet: 1 = the tracklet's ternary factor starts out
     of the graph (null: every ternary present, as in the reference). Lets a
     test restart the outlier_reject = 2 re-solve from any LM state. */
  const uint8_t* ternary_inactive;
} dynorefine_batch;

typedef struct {
  double landmark_motion_sigma; /* 0.001  (MotionSolver.hpp:217)            */
  double projection_sigma;      /* 2.0    (:218)                            */
  double k_huber;               /* 0.0001 (:219)                            */
  double prior_sigma;           /* 1e-5   (MotionSolver-inl.hpp:307)        */
  int outlier_reject;           /* 1 (:220); see above for 0 / 2            */
  int reserved;
} dynorefine_params;

enum { DYNOREFINE_OK = 0, DYNOREFINE_VALUES_KEY_EXISTS = 1 };

typedef struct {
  int iterations;        /* accepted LM iterations (all rounds)            */
  int inner_iterations;  /* linear solves (all rounds)                     */
  int status;            /* DYNOREFINE_*                                   */
  int n_outliers;        /* tracklets flagged                              */
  double error_before;   /* graph.error(values)                            */
  double error_after;    /* mutable_graph.error(optimised_values)          */
} dynorefine_result;

typedef struct dynorefine_solver dynorefine_solver;

void dynorefine_params_default(dynorefine_params* p);
int dynorefine_create(int device_id, dynorefine_solver** out);
void dynorefine_destroy(dynorefine_solver* s);
const char* dynorefine_last_error(const dynorefine_solver* s);

/* Upload a batch (copied; the device copy stays until the next upload). */
int dynorefine_upload(dynorefine_solver* s, const dynorefine_batch* b);
/* Solve every problem of the uploaded batch (one launch; the LM loops run on
   the device). Restarts from the uploaded initial values each call. */
int dynorefine_solve(dynorefine_solver* s, const dynorefine_params* p, const dynohip_lm_params* lm);
/* Results of the last solve: H (12 per problem), per-tracklet outlier flags
   and per-problem summaries. Any pointer may be null. */
int dynorefine_download(dynorefine_solver* s, double* H_out, uint8_t* outlier_out, dynorefine_result* results);
/* upload + solve + download */
int dynorefine_run(dynorefine_solver* s, const dynorefine_batch* b, const dynorefine_params* p,
                   const dynohip_lm_params* lm, double* H_out, uint8_t* outlier_out, dynorefine_result* results);
/* device time of the last solve (ms, HIP events on the launch stream) */
double dynorefine_last_solve_ms(const dynorefine_solver* s);

#ifdef __cplusplus
}
#endif

#endif /* DYNOREFINE_H_ */
