"""Regenerates the committed fixtures in tests/golden/.

1. ternary_perturbation.json: the 6-D tangent draw of perturbWithNoise(H, 0.3)
   with gtsam::Sampler seed 42 (sampler42.cpp, g++/libstdc++), and the
   inputs of test_factors.cc:143-203 (H = Rodrigues(-0.1, 0.2, 0.25),
   t = (0.05, -0.10, 0.20), P1 = (0.4, 1.0, 0.8)).
2. lm_T1.json / lm_T2.json: oracle LM traces + final values on the
   synthetic T1/T2 graphs (regression pins of the oracle itself).
"""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def sampler():
    with tempfile.TemporaryDirectory() as d:
        exe = os.path.join(d, "s42")
        subprocess.check_call(["g++", "-O0", "-o", exe, os.path.join(HERE, "sampler42.cpp")])
        out = subprocess.check_output([exe]).decode().split()
    return [float(x) for x in out]


def main():
    fx = {
        "source": "dynosam/test/test_factors.cc:143-203; GtsamUtils.hpp:202-219 (Sampler seed 42)",
        "H_rodrigues": [-0.1, 0.2, 0.25],
        "H_t": [0.05, -0.10, 0.20],
        "P1": [0.4, 1.0, 0.8],
        "perturb_sigma": 0.3,
        "perturb_tangent": sampler(),
        "noise_sigma": 0.1,
    }
    with open(os.path.join(HERE, "ternary_perturbation.json"), "w") as f:
        json.dump(fx, f, indent=1)
    from dynosam_amd import synth
    from oracle_binding import Oracle
    for name in ("T1", "T2"):
        g, v, _ = synth.generate(name)
        o = Oracle(g, v)
        s = o.optimize()
        out = {
            "config": name,
            "iterations": s.iterations,
            "inner_iterations": s.inner_iterations,
            "initial_error": s.initial_error,
            "final_error": s.final_error,
            "trace": o.trace(),
            "final_values": o.values_data().tolist(),
        }
        with open(os.path.join(HERE, f"lm_{name}.json"), "w") as f:
            json.dump(out, f)
    print("fixtures written")


if __name__ == "__main__":
    main()
