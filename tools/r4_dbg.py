"""Round-4 debug: a few LM iterations on small graphs with progress prints
(DYNOHIP_FUSED_LONE selects the static-landmark path)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynosam_amd import synth  # noqa: E402
from dynosam_amd.optimizer import Solver  # noqa: E402

for name in sys.argv[1:] or ["T1"]:
    g, v, _ = synth.generate(name)
    s = Solver(0)
    s.set_graph(g)
    s.set_values(v)
    print(name, "fused", os.environ.get("DYNOHIP_FUSED_LONE", "default"), "error", s.error(), flush=True)
    for it in range(3):
        t = time.time()
        sm = s.iterate()
        print(name, it, sm.iterations, sm.inner_iterations, sm.final_error, f"{(time.time() - t) * 1e3:.2f} ms", flush=True)
    s.close()
