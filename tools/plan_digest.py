"""Per-field digests of the host plan (dynohip_plan_export "digest") for a set
of graphs: `save PATH` writes them, `check PATH` compares against a saved set
and names the fields that differ. A planner refactor must leave every digest
unchanged. usage: python tools/plan_digest.py save|check PATH"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import plan_export  # noqa: E402

CASES = [("T2", {}, 1), ("T2", {"formulation": 1}, 1), ("C1", {}, 1), ("C2", {}, 1), ("C2", {}, 2),
         ("C1", {"formulation": 1}, 1), ("NS", {}, 1)]


def digests(suffix=""):
    from graphs_extra import mixed_lone_graph
    out = {}
    for name, kw, nr in CASES:
        g, v, _ = synth.generate(name, **kw)
        for r in range(nr):
            out["%s%s_r%d_of%d" % (name, "-ll" if kw else "", r, nr)] = plan_export(g, v, "digest" + suffix, nr, r)
    g, v, _, _ = mixed_lone_graph()
    out["mixed"] = plan_export(g, v, "digest" + suffix)
    return out


if __name__ == "__main__":
    mode, path = sys.argv[1], sys.argv[2]
    d = digests()
    if mode == "save":
        np.savez(path, **d)
        print("saved", len(d))
    else:
        ref = np.load(path)
        bad = 0
        for k, x in d.items():
            y = ref[k]
            if x.shape != y.shape or not np.array_equal(x, y):
                fields = np.nonzero((x.reshape(-1, 2) != y.reshape(-1, 2)).any(1))[0] if x.shape == y.shape else "shape"
                print("DIFF", k, fields)
                bad += 1
        print("ok" if not bad else "%d cases differ" % bad)
        sys.exit(1 if bad else 0)
