"""Summary of a rocprofv3 --kernel-trace of `bench.py --mode stream`:
kernel time per LM try (one try = one k_factor_persist launch), trace span,
busy fraction, and the GPU idle time between consecutive kernels split into
gaps inside window solves (< 1 ms: host decision / launch latency) and
longer ones (host graph construction and planning between solves).

usage: python tools/stream_summary.py <dir containing run_kernel_trace.csv>
"""
import csv
import glob
import sys
from collections import defaultdict


def short(name):
    n = name.replace("dynohip::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main(d):
    f = (glob.glob(d + "/**/run_kernel_trace.csv", recursive=True) or glob.glob(d + "/run_kernel_trace.csv"))[0]
    rows = list(csv.DictReader(open(f)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    tries = sum(1 for e in ev if e[2] == "k_factor_persist")
    span = (ev[-1][1] - ev[0][0]) / 1e6
    busy = sum(e[1] - e[0] for e in ev) / 1e6
    per = defaultdict(lambda: [0, 0.0])
    for s, e, n in ev:
        per[n][0] += 1
        per[n][1] += (e - s) / 1e3
    small = large = 0.0
    nsmall = 0
    end = ev[0][1]
    for s, e, n in ev[1:]:
        g = (s - end) / 1e3
        if g > 0:
            if g < 1000:
                small += g
                nsmall += 1
            else:
                large += g
        end = max(end, e)
    print(f"trace span {span:.1f} ms, kernel busy {busy:.1f} ms ({100 * busy / span:.0f}%), LM tries {tries}, "
          f"kernel time per try {1e3 * busy / max(tries, 1):.1f} us")
    print(f"idle gaps < 1 ms: {small / 1e3:.1f} ms in {nsmall} gaps ({small / max(tries, 1):.1f} us per try); "
          f"gaps >= 1 ms (host construction / planning): {large / 1e3:.1f} ms")
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1]):
        print(f"{n[:32]:32s} calls={c:6d} total_ms={t / 1e3:8.2f} avg_us={t / c:8.2f} per_try_us={t / max(tries, 1):7.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
