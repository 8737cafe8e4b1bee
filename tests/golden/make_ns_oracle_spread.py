"""Generates tests/golden/ns_oracle_spread.json: the CPU oracle's own
free-running LM trace on the north-star graph (synth "NS") in two summation
orders (oracle_set_reverse_sums off / on). The per-iteration difference of
the two traces is the spread any double-precision implementation of the same
LM shows on this graph from rounding alone; test_free_running_ns_vs_oracle
holds the GPU's distance to the oracle to it.

Run from the repository root: python tests/golden/make_ns_oracle_spread.py
(about two minutes on 8 cores)."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))

from dynosam_amd import synth  # noqa: E402
from oracle_binding import Oracle  # noqa: E402


def main():
    g, v, _ = synth.generate("NS")
    runs = {}
    for name, rev in (("forward", False), ("reversed", True)):
        o = Oracle(g, v, threads=min(8, os.cpu_count() or 1), reverse_sums=rev)
        r = o.optimize()
        runs[name] = {
            "iterations": r.iterations,
            "inner_iterations": r.inner_iterations,
            "final_error": r.final_error,
            "trace": [{"lam": e["lam"], "accepted": int(e["accepted"]), "new_error": e["new_error"]}
                      for e in o.trace()],
        }
    out = os.path.join(HERE, "ns_oracle_spread.json")
    with open(out, "w") as f:
        json.dump(runs, f, indent=1)
    print("wrote", out)


if __name__ == "__main__":
    main()
