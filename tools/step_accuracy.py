"""Accuracy of the damped LM step at deep convergence.
Along the oracle's own LM run on a synthetic config, at every iteration's
first lambda, the step of:
  oracle     the CPU restatement (double, Schur + envelope Cholesky),
  reversed   the same with its sums in reverse order (rounding control),
  gpu        dynohip_solve_delta on the same values (--gpu, needs the GPU),
against the step with the Schur solve in x87 extended precision
(oracle_solve_damped_ld, eps 5.4e-20). Printed relative to the values'
norm (the per-iteration parity metric) and to the reference step's norm.
usage: python tools/step_accuracy.py [C2] [iters] [--gpu]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import _abi, synth  # noqa: E402
from oracle_binding import Oracle  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
name = args[0] if args else "C2"
iters = int(args[1]) if len(args) > 1 else 15
gpu = "--gpu" in sys.argv
g, v, _ = synth.generate(name)
o = Oracle(g, v)
r = Oracle(g, v, reverse_sums=True)
s = None
if gpu:
    from dynosam_amd.optimizer import Solver
    s = Solver(0)
    s.set_graph(g)
    s.set_values(v)
p = _abi.LMParams.gtsam_default()
lam = 1e-5
o.reset(p)
for it in range(iters):
    # the run follows the GPU's iterates when it is there (as the
    # conditioned parity test does), else the oracle's
    data = s.values_data() if s is not None else o.values_data()
    o.set_values_data(data)
    r.set_values_data(data)
    vn = np.linalg.norm(data)
    ok_l, dl = o.solve_damped_ld(lam)
    ok_o, do = o.solve_damped(lam)
    ok_r, dr = r.solve_damped(lam)
    line = [f"{name} {it} lambda {lam:.0e}", f"|step|/|values| {np.linalg.norm(dl) / vn:.2e}"]
    for tag, d, ok in (("oracle", do, ok_o), ("reversed", dr, ok_r)):
        line.append(f"{tag} {np.linalg.norm(d - dl) / vn:.2e} ({np.linalg.norm(d - dl) / np.linalg.norm(dl):.1e})"
                    if ok and ok_l else f"{tag} fail")
    if s is not None:
        ok_g, dg = s.solve_delta(lam)   # the GPU is on `data` (it drives the run)
        line.append(f"gpu {np.linalg.norm(dg - dl) / vn:.2e} ({np.linalg.norm(dg - dl) / np.linalg.norm(dl):.1e})"
                    if ok_g and ok_l else "gpu fail")
        line.append(f"gpu-oracle {np.linalg.norm(dg - do) / vn:.2e}")
    print("  ".join(line), flush=True)
    p.lambda_initial = lam
    if s is not None:
        s.reset(p)
        lam = s.iterate().final_lambda
    else:
        o.reset(p)
        lam = o.iterate().final_lambda
