"""Rounding control for the deep-convergence parity: the CPU
oracle against itself with the Schur solve's sums reversed (the same
mathematics, other rounding; oracle_set_reverse_sums), conditioned per LM
iteration exactly as tests/test_gpu_parity.py conditions the GPU: before
every iteration both copies are put on the same values and lambda.
usage: python tools/rounding_control.py [C2] [iters]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import _abi, synth  # noqa: E402
from oracle_binding import Oracle  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 15
g, v, _ = synth.generate(name)
a = Oracle(g, v)                       # the reference sums
b = Oracle(g, v, reverse_sums=True)   # reversed sums
lam = 1e-5
p = _abi.LMParams.gtsam_default()
for it in range(iters):
    start = a.values_data()
    b.set_values_data(start)
    p.lambda_initial = lam
    a.reset(p)
    b.reset(p)
    sa, sb = a.iterate(), b.iterate()
    va, vb = a.values_data(), b.values_data()
    vr = np.linalg.norm(va - vb) / np.linalg.norm(va)
    er = abs(sa.final_error - sb.final_error) / abs(sa.final_error)
    print(f"{name} {it} lambda {lam:.0e} tries {sa.inner_iterations}/{sb.inner_iterations} "
          f"values rel {vr:.2e} error rel {er:.2e}", flush=True)
    lam = sa.final_lambda
