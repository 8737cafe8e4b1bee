/*
 * dynosynth.h — deterministic synthetic DynoSAM backend graphs (C-ABI).
 *
 * Mirrors the factor-graph structure the reference WorldMotion formulation
 * builds with do_backtrack = false:
 *   - X_k camera poses, prior on X_0 (Formulation-impl.hpp:91-104),
 *     odometry Between from the frontend poses (Formulation-impl.hpp:133-156);
 *   - static points l_i: L_s consecutive observations, the first dropped
 *     (min_static_obs = 2, Formulation-impl.hpp:245-291), initialised from
 *     the frontend pose at the frame the point enters;
 *   - dynamic tracklets: L_d observations, points m_{i,k} from the second
 *     observation on (min_dynamic_obs = 3, WorldMotionEstimator.cc:155-238),
 *     PoseToPoint per point, LandmarkMotionTernary per consecutive pair,
 *     H_{j,k} initialised to identity (init_H_with_identity,
 *     WorldMotionEstimator.cc:260-266), smoothing Between(H_{k-1}, H_k, I)
 *     (WorldMotionEstimator.cc:271-301).
 * Noise: the shipped backend.flags (default) or BackendParams code defaults.
 * RNG: std::mt19937_64(seed) + in-repo Box–Muller, so every consumer gets
 * bit-identical graphs.
 *
 * Also generates the LLWorld (WorldPose) variant: object poses L_{j,k}
 * with LandmarkMotionPose and LandmarkPoseSmoothing factors
 * (WorldPoseEstimator.cc:84-286).
 */
#ifndef DYNOSYNTH_H_
#define DYNOSYNTH_H_

#include <stddef.h>
#include <stdint.h>

#include "dynohip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int frames;              /* F                                           */
  int objects;             /* O                                           */
  int static_landmarks;    /* S                                           */
  int dyn_slots;           /* P_dyn concurrent tracklets per object       */
  int static_track_len;    /* L_s (default 8)                             */
  int dyn_track_len;       /* L_d (default 10)                            */
  uint64_t seed;           /* 42                                          */
  int noise_code_defaults; /* 0: backend.flags, 1: BackendParams defaults  */
  int object_visible_frames; /* 0: all frames, else window length         */
  int formulation;         /* 0: MotionInWorld, 1: LLWorld                 */
  int smoothing;           /* 1: add motion smoothing factors             */
  int robust;              /* 1: Huber on point / motion factors          */
} dynosynth_config;

typedef struct dynosynth dynosynth;

void dynosynth_config_default(dynosynth_config* c);
int dynosynth_generate(const dynosynth_config* c, dynosynth** out);
void dynosynth_destroy(dynosynth* s);
/* pointers stay valid until dynosynth_destroy */
void dynosynth_graph(const dynosynth* s, dynohip_graph_view* g);
size_t dynosynth_num_values(const dynosynth* s);
size_t dynosynth_values_len(const dynosynth* s);
const uint64_t* dynosynth_value_keys(const dynosynth* s);
const uint8_t* dynosynth_value_kinds(const dynosynth* s);
const double* dynosynth_value_data(const dynosynth* s);
/* ground truth in the same layout as value data */
const double* dynosynth_ground_truth(const dynosynth* s);

#ifdef __cplusplus
}
#endif

#endif
