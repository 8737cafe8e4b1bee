"""Per-phase minimum over the reps of a DYNOHIP_PLAN_TIMING / SCHED_TIMING
log (tools/plan_timing.py output). usage: python tools/plan_phase_min.py LOG..."""
import re
import sys

for path in sys.argv[1:]:
    best, order = {}, []
    for line in open(path):
        m = re.match(r"\s*(\[plan\]|\[tiles\]|csr/src|csr)\s*(.*?)\s+([0-9.]+) ms\s*$", line)
        if m and m.group(1) in ("[plan]", "[tiles]"):
            key = m.group(1) + " " + m.group(2)
            v = float(m.group(3))
        else:
            m = re.match(r"\s*(csr(?:/src)?) (nt=\d+) .*count ([0-9.]+)(?: alloc [0-9.]+)? fill ([0-9.]+) ms", line)
            if not m:
                continue
            key = "%s %s" % (m.group(1), m.group(2))
            v = float(m.group(3)) + float(m.group(4))
        if key not in best:
            order.append(key)
            best[key] = v
        best[key] = min(best[key], v)
    print("==", path)
    for k in order:
        print("%-64s %7.2f" % (k, best[k]))
