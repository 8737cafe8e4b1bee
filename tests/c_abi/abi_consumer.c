/*
 * abi_consumer.c — a plain C99 caller of include/dynohip.h, compiled with gcc
 * (no C++ and no Python between it and the library), pinning the C-ABI
 * outside ctypes.
 *
 *   abi_consumer host   host-only entry points: ABI version, LM defaults
 *                       (GTSAM LevenbergMarquardtParams), keys
 *                       (DynamicPointSymbol.cc:31-44, BackendDefinitions.hpp),
 *                       SlidingWindow::check (RGBDBackendModule.hpp:120-144,
 *                       incl. the CHECK_GE as DYNOHIP_EINVAL), the full-batch
 *                       trigger, and that dynohip_create fails cleanly without
 *                       a device.
 *   abi_consumer gpu    the T2 graph (libdynosynth) through
 *                       create/set_graph/set_values/optimize/get_values on
 *                       device 0, checked against the CPU oracle
 *                       (liboracle.so, test infrastructure): same iterations
 *                       and inner iterations, values within 1e-6 relative;
 *                       then one dynorefine batch with every field of the
 *                       version-3 dynorefine_batch filled (incl. the
 *                       trailing ternary_inactive mask): an all-zero mask
 *                       gives the same results as a null one.
 *
 * Prints "OK ..." and exits 0 on success; any mismatch exits 1.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "dynohip.h"
#include "dynorefine.h"
#include "dynosynth.h"
#include "oracle.h"

static int fails = 0;
#define EXPECT(c, ...)                                 \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fputc('\n', stderr);                             \
      ++fails;                                         \
    }                                                  \
  } while (0)

static int host_checks(void) {
  dynohip_lm_params p;
  dynohip_solver* s = NULL;
  dynohip_sliding_window w;
  uint64_t start = 0;
  uint64_t k1 = 0, k2 = 0;
  EXPECT(dynohip_abi_version() == DYNOHIP_ABI_VERSION, "abi version %d", dynohip_abi_version());
  dynohip_lm_params_default(&p);
  EXPECT(p.max_iterations == 100, "max_iterations %d", p.max_iterations);
  EXPECT(p.lambda_initial == 1e-5 && p.lambda_factor == 10.0, "lambda %g %g", p.lambda_initial, p.lambda_factor);
  EXPECT(p.relative_error_tol == 1e-5 && p.absolute_error_tol == 1e-5, "tols");
  /* CameraPoseSymbol(7) = gtsam::Symbol(kPosesSymbolChar, 7) */
  EXPECT(dynohip_symbol_index(dynohip_camera_pose_key(7)) == 7, "camera key index");
  EXPECT(dynohip_chr_extract(dynohip_camera_pose_key(7)) == dynohip_symbol_chr(dynohip_camera_pose_key(7)),
         "camera key chr");
  EXPECT(dynohip_symbol_index(dynohip_symbol('l', 42)) == 42, "symbol index");
  EXPECT(dynohip_symbol_chr(dynohip_symbol('l', 42)) == 'l', "symbol chr");
  /* Cantor pairing round trip, incl. the reference test's tracklet 46528 */
  dynohip_cantor_depair(dynohip_cantor_pair(46528, 12), &k1, &k2);
  EXPECT(k1 == 46528 && k2 == 12, "cantor %llu %llu", (unsigned long long)k1, (unsigned long long)k2);
  /* SlidingWindow(window 10, overlap 4) from frame 0: the first window is
     [0, 10], triggered at frame 10 (previous_trigger_frame starts at 4) */
  dynohip_sliding_window_init(&w, 10, 4);
  {
    int rc = 0;
    uint64_t k, end = 0;
    for (k = 0; k < 10 && rc == 0; ++k) rc = dynohip_sliding_window_check(&w, k, &start, &end);
    EXPECT(rc == 0, "no trigger before frame 10 (rc %d)", rc);
    rc = dynohip_sliding_window_check(&w, 10, &start, &end);
    EXPECT(rc == 1 && start == 0 && end == 10, "trigger at 10: rc %d [%llu, %llu]", rc, (unsigned long long)start,
           (unsigned long long)end);
    /* next window [6, 16] (overlap 4) */
    for (k = 11; k < 16 && rc >= 0; ++k) rc = dynohip_sliding_window_check(&w, k, &start, &end);
    rc = dynohip_sliding_window_check(&w, 16, &start, &end);
    EXPECT(rc == 1 && start == 6, "trigger at 16: rc %d start %llu", rc, (unsigned long long)start);
  }
  /* CHECK_GE(starting_frame, first_frame) -> DYNOHIP_EINVAL: window 3,
     overlap 5, first frame 10; triggers at 13, then frame 11 would start
     a window at 8 < 10 */
  dynohip_sliding_window_init(&w, 3, 5);
  {
    uint64_t k;
    int rc = 0;
    for (k = 10; k < 14; ++k) rc = dynohip_sliding_window_check(&w, k, &start, NULL);
    EXPECT(rc == 1 && start == 10, "trigger at 13: rc %d start %llu", rc, (unsigned long long)start);
    rc = dynohip_sliding_window_check(&w, 11, &start, NULL);
    EXPECT(rc == DYNOHIP_EINVAL, "window before the first frame: rc %d", rc);
  }
  /* first frame beyond INT_MAX (CHECK_GE(first_frame, 0)) */
  dynohip_sliding_window_init(&w, 10, 4);
  EXPECT(dynohip_sliding_window_check(&w, (uint64_t)1 << 31, &start, NULL) == DYNOHIP_EINVAL, "first frame > INT_MAX");
  /* RGBDBackendModule.cc:201-202: full batch at frame full_batch_frame - 1 */
  EXPECT(dynohip_full_batch_trigger(6, 5) == 1, "full batch at its frame");
  EXPECT(dynohip_full_batch_trigger(6, 6) == 0, "full batch only once");
  /* dynorefine_batch layout of this header version (13 pointer-sized fields) */
  EXPECT(sizeof(dynorefine_batch) == 13 * sizeof(void*), "dynorefine_batch size %zu", sizeof(dynorefine_batch));
  /* no device in the build container: create reports an error, no crash */
  if (getenv("ABI_EXPECT_NO_DEVICE")) {
    int rc = dynohip_create(0, &s);
    EXPECT(rc != DYNOHIP_OK && s == NULL, "create without a device: rc %d", rc);
  }
  return fails;
}

/* one (object, frame pair) refinement problem, 12 tracklets of a rigid body
   moved by a small motion and seen by a camera that moved too */
static int refine_checks(void) {
  enum { NT = 12 };
  double Xa[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0}, Xb[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0.1, 0, 0};
  double H0[12] = {1, 0, 0, 0, 1, 0, 0, 0, 1, 0, 0, 0}, cal[5] = {500, 500, 0, 320, 240};
  double kpa[2 * NT], kpb[2 * NT], ma[3 * NT], mb[3 * NT], Ha[12], Hb[12];
  int32_t ts[2] = {0, NT};
  uint8_t mask[NT], oa[NT], ob[NT];
  dynorefine_result ra, rb;
  dynorefine_params rp;
  dynohip_lm_params lm;
  dynorefine_batch b;
  dynorefine_solver* r = NULL;
  int i, k, bad = 0;
  for (i = 0; i < NT; ++i) {
    const double x = -0.5 + 0.09 * i, y = 0.3 * ((i % 3) - 1), z = 4.0 + 0.05 * (i % 5);
    ma[3 * i] = x; ma[3 * i + 1] = y; ma[3 * i + 2] = z;
    mb[3 * i] = x + 0.05; mb[3 * i + 1] = y; mb[3 * i + 2] = z + 0.02; /* true motion: a translation */
    kpa[2 * i] = cal[0] * x / z + cal[3];
    kpa[2 * i + 1] = cal[1] * y / z + cal[4];
    kpb[2 * i] = cal[0] * (mb[3 * i] - Xb[9]) / mb[3 * i + 2] + cal[3];
    kpb[2 * i + 1] = cal[1] * mb[3 * i + 1] / mb[3 * i + 2] + cal[4];
    mask[i] = 0;
  }
  memset(&b, 0, sizeof(b));
  b.n_problems = 1;
  b.track_start = ts;
  b.X_k_1 = Xa;
  b.X_k = Xb;
  b.H_init = H0;
  b.calibration = cal;
  b.kp_k_1 = kpa;
  b.kp_k = kpb;
  b.m_k_1 = ma;
  b.m_k = mb;
  b.X_k_1_init = Xa;
  b.X_k_init = Xb;
  b.ternary_inactive = NULL;
  dynorefine_params_default(&rp);
  dynohip_lm_params_default(&lm);
  if (dynorefine_create(0, &r) != DYNOHIP_OK) return 1;
  if (dynorefine_run(r, &b, &rp, &lm, Ha, oa, &ra) != DYNOHIP_OK) {
    fprintf(stderr, "dynorefine: %s\n", dynorefine_last_error(r));
    dynorefine_destroy(r);
    return 1;
  }
  b.ternary_inactive = mask;
  if (dynorefine_run(r, &b, &rp, &lm, Hb, ob, &rb) != DYNOHIP_OK) {
    fprintf(stderr, "dynorefine (mask): %s\n", dynorefine_last_error(r));
    dynorefine_destroy(r);
    return 1;
  }
  for (k = 0; k < 12; ++k) bad += !isfinite(Ha[k]) || Ha[k] != Hb[k];
  for (i = 0; i < NT; ++i) bad += oa[i] != ob[i];
  bad += ra.iterations != rb.iterations || ra.inner_iterations != rb.inner_iterations || ra.status != rb.status;
  bad += !(ra.error_after <= ra.error_before);
  if (bad) fprintf(stderr, "dynorefine: masked/unmasked mismatch (%d)\n", bad);
  dynorefine_destroy(r);
  return bad;
}

static int gpu_checks(void) {
  dynosynth_config c;
  dynosynth* g = NULL;
  dynohip_graph_view view;
  dynohip_solver* s = NULL;
  oracle_problem* o = NULL;
  dynohip_lm_params p;
  dynohip_lm_summary gs, os;
  size_t n, len, i;
  double *gv = NULL, *ov = NULL, num = 0.0, den = 0.0;

  dynosynth_config_default(&c);
  c.frames = 20; /* the T2 graph of dynosam_amd/synth.py */
  c.objects = 2;
  c.static_landmarks = 120;
  c.dyn_slots = 4;
  if (dynosynth_generate(&c, &g) != 0) { fprintf(stderr, "synth failed\n"); return 1; }
  dynosynth_graph(g, &view);
  n = dynosynth_num_values(g);
  len = dynosynth_values_len(g);
  dynohip_lm_params_default(&p);

  if (dynohip_create(0, &s) != DYNOHIP_OK) { fprintf(stderr, "create failed\n"); return 1; }
  if (dynohip_set_graph(s, &view) != DYNOHIP_OK ||
      dynohip_set_values(s, dynosynth_value_keys(g), dynosynth_value_kinds(g), dynosynth_value_data(g), n) != DYNOHIP_OK ||
      dynohip_optimize(s, &p, &gs) != DYNOHIP_OK) {
    fprintf(stderr, "dynohip: %s\n", dynohip_last_error(s));
    return 1;
  }
  gv = (double*)malloc(len * sizeof(double));
  ov = (double*)malloc(len * sizeof(double));
  EXPECT(dynohip_get_values(s, gv, len) == DYNOHIP_OK, "get_values");

  if (oracle_create(&view, dynosynth_value_keys(g), dynosynth_value_kinds(g), dynosynth_value_data(g), n, &o) != 0 ||
      oracle_optimize(o, &p, &os) != 0) {
    fprintf(stderr, "oracle failed\n");
    return 1;
  }
  oracle_get_values(o, ov, len);
  for (i = 0; i < len; ++i) {
    num += (gv[i] - ov[i]) * (gv[i] - ov[i]);
    den += ov[i] * ov[i];
  }
  EXPECT(gs.iterations == os.iterations, "iterations %d vs %d", gs.iterations, os.iterations);
  EXPECT(gs.inner_iterations == os.inner_iterations, "inner %d vs %d", gs.inner_iterations, os.inner_iterations);
  EXPECT(sqrt(num / den) < 1e-6, "values rel %.3e", sqrt(num / den));
  EXPECT(fabs(gs.final_error - os.final_error) <= 1e-6 * fabs(os.final_error), "final error %.9g vs %.9g",
         gs.final_error, os.final_error);
  EXPECT(refine_checks() == 0, "dynorefine batch");
  printf("OK gpu iterations=%d inner=%d rel=%.3e error=%.9g\n", gs.iterations, gs.inner_iterations, sqrt(num / den),
         gs.final_error);
  free(gv);
  free(ov);
  oracle_destroy(o);
  dynohip_destroy(s);
  dynosynth_destroy(g);
  return fails;
}

int main(int argc, char** argv) {
  int rc;
  if (argc < 2) { fprintf(stderr, "usage: %s host|gpu\n", argv[0]); return 2; }
  if (strcmp(argv[1], "host") == 0) {
    rc = host_checks();
    if (rc == 0) printf("OK host\n");
    return rc ? 1 : 0;
  }
  if (strcmp(argv[1], "gpu") == 0) return gpu_checks() ? 1 : 0;
  return 2;
}
