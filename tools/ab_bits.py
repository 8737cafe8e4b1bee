"""A/B bit comparison of two builds (speed-only changes must not move a bit).
  python tools/ab_bits.py run <out.npz> [configs...]   (DYNOSAM_AMD_LIB_DIR picks the build)
  python tools/ab_bits.py cmp <a.npz> <b.npz>
`run` records, per config, one damped solve at lambda 1e-3 (the step, in value
order) and a full LM run (final values and the per-iteration trace).
The round-4 comparisons (tools/r4_gred*.sh) ran against variants/old, the
build of commit 7944cfa: `git archive 7944cfa dynosam_amd/csrc include | tar -x
-C /tmp/old` and the hipcc line of tools/build_variant.sh run there, output
into variants/old (git-ignored)."""
import sys

import numpy as np

sys.path.insert(0, ".")


def run(out, names):
    from dynosam_amd import synth
    from dynosam_amd.optimizer import Solver
    res = {}
    for name in names:
        g, v, _ = synth.generate(name)
        s = Solver(0)
        s.set_graph(g)
        s.set_values(v)
        ok, d = s.solve_delta(1e-3)
        res[name + "/delta"] = d
        res[name + "/delta_ok"] = np.array([ok])
        s.set_values(v)
        r = s.optimize()
        res[name + "/values"] = s.values_data()
        tr = s.trace()
        res[name + "/trace"] = np.array([[float(e[k]) for k in sorted(e)] for e in tr]) if tr else np.zeros((0, 0))
        res[name + "/iters"] = np.array([r.iterations])
        s.close()
        print(name, "iterations", r.iterations, flush=True)
    np.savez(out, **res)


def cmp(a, b):
    A, B = np.load(a), np.load(b)
    bad = 0
    for k in sorted(A.files):
        x, y = A[k], B[k]
        same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
        if not same:
            bad += 1
            diff = np.abs(x - y).max() if x.shape == y.shape else float("nan")
            print("DIFF", k, x.shape, y.shape, "max abs diff", diff)
        else:
            print("same", k, x.shape)
    print("bit-identical" if bad == 0 else "%d arrays differ" % bad)
    return bad


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3:] or ["C1", "C2", "NS"])
    else:
        sys.exit(1 if cmp(sys.argv[2], sys.argv[3]) else 0)
