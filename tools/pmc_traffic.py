"""Summarise two rocprofv3 PMC passes (tools/pmc_pass.sh: FETCH_SIZE, then
WRITE_SIZE, each its own run of the same bench command) into per-launch HBM
traffic per kernel and per factorisation.

Corrections follow /opt/skills/guides/MI355X_MICROARCH.md (HBM section):
  FETCH_SIZE and WRITE_SIZE are KB per dispatch. On gfx950, FETCH_SIZE
  reports half the bytes of wide (16 B/lane) coalesced reads, so it is
  doubled here. WRITE_SIZE is taken as is. Other access widths are
  uncalibrated, and the raw values are kept next to the corrected ones.
  Infinity-Cache hits are counted, not excluded.

usage: python tools/pmc_traffic.py <pmc dir> <config> <out.json>
"""
import csv
import json
import sys
from collections import defaultdict


def load(path):
    per = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        short = name.replace("dynohip::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        per[short].append(float(r["Counter_Value"]) * 1024.0)
    return per


def main():
    d, config, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch = load(f"{d}/FETCH_SIZE_counter_collection.csv")
    write = load(f"{d}/WRITE_SIZE_counter_collection.csv")
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        f, w = fetch.get(k, []), write.get(k, [])
        n = max(len(f), len(w))
        kernels[k] = {
            "dispatches": n,
            "fetch_raw_bytes_per_launch": sum(f) / max(len(f), 1),
            "write_bytes_per_launch": sum(w) / max(len(w), 1),
            "traffic_bytes_per_launch": 2.0 * sum(f) / max(len(f), 1) + sum(w) / max(len(w), 1),
        }
    # one damped solve = one k_gather_band dispatch; the factorisation is the
    # k_tasks (+ k_updates) levels and the backward launch(es) of that solve
    nsolve = kernels.get("k_gather_band", {}).get("dispatches", 0)
    fac = None
    if nsolve:
        tot = 0.0
        for k in ("k_tasks", "k_updates", "k_back", "k_back_persist"):
            if k in kernels:
                tot += kernels[k]["traffic_bytes_per_launch"] * kernels[k]["dispatches"]
        fac = tot / nsolve
    res = {"config": config, "solves": nsolve, "traffic_bytes_per_factorisation": fac, "kernels": kernels,
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs, --kernel-trace); "
                     "bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction, MI355X_MICROARCH.md HBM)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: round(v["traffic_bytes_per_launch"] / 1e6, 3) for k, v in kernels.items()}, indent=0))
    print("per factorisation MB:", fac / 1e6 if fac else None)


if __name__ == "__main__":
    main()
