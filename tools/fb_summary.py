"""min / median of each stage over the calls of a tools/fb_timing.py log
(persistent-handle calls and fresh-handle calls after the first).
usage: python tools/fb_summary.py LOG [label]"""
import re
import statistics
import sys

vals = {}
fresh = True
first = True
for line in open(sys.argv[1]):
    if line.startswith("persistent"):
        fresh = False
    m = re.match(r"\w+ (.*) total=([0-9.]+) ms", line)
    if not m:
        continue
    if fresh and first:
        first = False
        continue
    for k, v in re.findall(r"(\w+)=([0-9.]+)", m.group(1)):
        vals.setdefault(("fresh " if fresh else "pers ") + k, []).append(float(v))
    vals.setdefault(("fresh " if fresh else "pers ") + "total", []).append(float(m.group(2)))
label = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
print(label, " ".join("%s=%.2f/%.2f" % (k, min(v), statistics.median(v)) for k, v in vals.items()
                      if k.split()[1] in ("set_values", "total")))
