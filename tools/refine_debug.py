import sys, numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
import refine as orf
from dynosam_amd import refine
from test_refine import _shift_every_fifth
batch = refine.synthetic_batch(12, tracks=(10, 40), seed=5, outlier_frac=0.15)
batch.kp_k = _shift_every_fifth(batch)
params = dict(landmark_motion_sigma=0.01, projection_sigma=0.5, outlier_reject=2)
opt = refine.MotionOnlyRefinementOptimizer(**params)
H, flags, res = opt.optimize_batch(batch)
R = orf.Refiner(schur=True, **params)
for p in range(batch.n):
    d = batch.problem(p)
    pb = orf.Problem(d["X_k_1"], d["X_k"], d["H"], d["K"], d["kp_k_1"], d["kp_k"], d["m_k_1"], d["m_k"])
    r = R.refine(pb)
    a, b = batch.track_start[p], batch.track_start[p+1]
    g = sorted(np.nonzero(flags[a:b])[0].tolist())
    Href = orf.p12(r["state"][2])
    print(p, res[p]["iterations"], r["iterations"], g == sorted(r["outliers"]), g, sorted(r["outliers"]), round(np.linalg.norm(H[p]-Href)/np.linalg.norm(Href), 8))
