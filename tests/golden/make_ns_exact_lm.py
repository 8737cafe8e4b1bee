"""Writes tests/golden/ns_exact_lm.npz: the north-star graph NS (500
frames, 5 objects, 100k landmarks; synth.generate("NS")) solved by the CPU
oracle's LM with every damped solve in x87 extended precision
(oracle_set_solve_ld: the exact-step trajectory), its final values, its
accept / lambda trace and its iteration counts. The deep-convergence free
run of tests/test_gpu_parity.py is compared with it (the double-precision
oracle stops two iterations early there, its last steps 6-50 % off the
exact ones). Serial, about two minutes. Run from the repository root after
`make -C oracle`: python tests/golden/make_ns_exact_lm.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from dynosam_amd import synth  # noqa: E402
from oracle_binding import Oracle  # noqa: E402


def main():
    g, v, _ = synth.generate("NS")
    o = Oracle(g, v, solve_ld=True)
    s = o.optimize()
    tr = o.trace()
    np.savez(os.path.join(ROOT, "tests", "golden", "ns_exact_lm.npz"), values=o.values_data(),
             iterations=s.iterations, inner_iterations=s.inner_iterations, final_error=s.final_error,
             lam=np.array([e["lam"] for e in tr]), accepted=np.array([e["accepted"] for e in tr]),
             new_error=np.array([e["new_error"] for e in tr]))
    print("NS exact-step LM:", s.iterations, s.inner_iterations, s.final_error)


if __name__ == "__main__":
    main()
