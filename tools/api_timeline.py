"""Host timeline of one sliding-window solve from a rocprofv3
--hip-trace --kernel-trace run of `bench.py --mode stream`: every HIP API
call (start relative to the window's plan-upload kernel, duration) and the
GPU kernels, merged in time order, plus per-API totals over all windows.

usage: python tools/api_timeline.py <trace dir> [window index]
"""
import csv
import glob
import sys
from collections import defaultdict


def short(n):
    n = n.replace("dynohip::(anonymous namespace)::", "").replace("dynohip::", "").replace("void ", "")
    return n.split("(")[0]


def load(d, name):
    f = (glob.glob(f"{d}/**/run_{name}.csv", recursive=True) or glob.glob(f"{d}/run_{name}.csv"))[0]
    return list(csv.DictReader(open(f)))


def main(d, w):
    api = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in load(d, "hip_api_trace")]
    ker = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "  [GPU] " + short(r["Kernel_Name"]))
           for r in load(d, "kernel_trace")]
    scat = sorted(k[0] for k in ker if "k_scatter_chunks" in k[2])
    t0, t1 = scat[w], scat[w + 1]
    # from a little before this window's plan upload to the next one
    lo = t0 - 3_000_000
    ev = sorted(e for e in api + ker if lo <= e[0] < t1)
    prev_end = None
    for s, e, n in ev:
        if n.startswith("  [GPU]") or (e - s) > 20_000 or n.startswith("hipLaunch") is False:
            print(f"{(s - t0) / 1e3:9.1f} us  {(e - s) / 1e3:8.1f} us  {n}")
        prev_end = e
    tot = defaultdict(lambda: [0, 0.0])
    for s, e, n in api:
        tot[n][0] += 1
        tot[n][1] += (e - s) / 1e3
    print("\nAPI totals over the run:")
    for n, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"{n:32s} calls={c:7d} total_ms={t / 1e3:8.2f} avg_us={t / c:7.2f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 10)
