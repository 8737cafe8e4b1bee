"""Per-kernel, per-launch HBM traffic and FP64 MFMA activity from rocprofv3
PMC passes of one bench command (tools/pmc_passes.sh), joined with the
kernel-trace durations of an unprofiled-counter run of the same command.

Passes (one rocprofv3 run each, --kernel-trace only, never with sys/runtime
trace domains; counter limits per pass: MI355X_MICROARCH.md "rocprofv3 PMC
slots"):
  fetch:  FETCH_SIZE                       (TCC: 3 of 4 slots)
  write:  WRITE_SIZE                       (TCC: 2 slots)
  mfma:   SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES
          SQ_INSTS_VALU_MFMA_F64 + GRBM_GUI_ACTIVE
Corrections (MI355X_MICROARCH.md, HBM): FETCH_SIZE and WRITE_SIZE are KB
per dispatch; on gfx950 FETCH_SIZE reports half the bytes of wide (16 B per
lane) coalesced reads, so it is doubled; WRITE_SIZE is taken as is. Other
access widths are uncalibrated: the raw values are kept beside the
corrected ones. Infinity-Cache hits are counted, not excluded.
MFMA: SQ_INSTS_VALU_MFMA_MOPS_F64 counts FP64 matrix work in units of 512
flops (rocprofv3's MfmaFlopsF64 = MOPS_F64 * 512); busy fraction =
SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 256 CUs x 4 SIMDs).

usage: python tools/pmc_summary.py <dir with fetch/ write/ mfma/ trace/> <config> <out.json>
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    n = name.replace("dynohip::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def counters(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return {}
    per = defaultdict(lambda: defaultdict(dict))   # kernel -> dispatch -> counter -> value
    for r in csv.DictReader(open(f[0])):
        per[short(r["Kernel_Name"])][r.get("Dispatch_Id", r.get("Correlation_Id", ""))][r["Counter_Name"]] = \
            float(r["Counter_Value"])
    return per


def durations(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    out = {}
    if f:
        for r in csv.DictReader(open(f[0])):
            out[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                     "pct": float(r["Percentage"])}
    return out


def mean(per_dispatch, ctr):
    v = [c[ctr] for c in per_dispatch.values() if ctr in c]
    return sum(v) / len(v) if v else None


def main():
    d, config, out = sys.argv[1], sys.argv[2], sys.argv[3]
    fetch, write, mfma = counters(f"{d}/fetch"), counters(f"{d}/write"), counters(f"{d}/mfma")
    dur = durations(f"{d}/trace")
    kernels = {}
    for k in sorted(set(fetch) | set(write) | set(mfma) | set(dur)):
        e = {"dispatches_profiled": len(fetch.get(k, {}))}
        if k in dur:
            e.update({"calls": dur[k]["calls"], "avg_us": dur[k]["avg_ns"] / 1e3, "time_pct": dur[k]["pct"]})
        f = mean(fetch.get(k, {}), "FETCH_SIZE")
        w = mean(write.get(k, {}), "WRITE_SIZE")
        if f is not None:
            e["fetch_raw_bytes_per_launch"] = f * 1024.0
        if w is not None:
            e["write_bytes_per_launch"] = w * 1024.0
        if f is not None and w is not None:
            e["traffic_bytes_per_launch"] = 2.0 * f * 1024.0 + w * 1024.0
            if "avg_us" in e and e["avg_us"] > 0:
                e["traffic_GBps"] = e["traffic_bytes_per_launch"] / (e["avg_us"] * 1e-6) / 1e9
        m = mfma.get(k)
        if m:
            mops = mean(m, "SQ_INSTS_VALU_MFMA_MOPS_F64")
            busy = mean(m, "SQ_VALU_MFMA_BUSY_CYCLES")
            gui = mean(m, "GRBM_GUI_ACTIVE")
            e["mfma_f64_flops_per_launch"] = mops * 512.0 if mops is not None else None
            e["mfma_f64_insts_per_launch"] = mean(m, "SQ_INSTS_VALU_MFMA_F64")
            e["mfma_busy_cycles_per_launch"] = busy
            e["grbm_gui_active_per_launch"] = gui
            if busy is not None and gui:
                e["mfma_busy_frac"] = busy / (gui / 8.0 * 256 * 4)
            if mops is not None and "avg_us" in e and e["avg_us"] > 0:
                e["mfma_f64_TFLOPs"] = mops * 512.0 / (e["avg_us"] * 1e-6) / 1e12
        kernels[k] = e
    res = {"config": config, "kernels": kernels,
           "method": "rocprofv3 --kernel-trace --stats (durations) and separate --pmc passes FETCH_SIZE | WRITE_SIZE | "
                     "SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 "
                     "GRBM_GUI_ACTIVE; bytes = 2*FETCH_SIZE + WRITE_SIZE (gfx950 correction, MI355X_MICROARCH.md); "
                     "MFMA flops = MOPS_F64 * 512"}
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    for k, e in sorted(kernels.items(), key=lambda kv: -kv[1].get("time_pct", 0))[:14]:
        print(f"{k[:34]:34s} us={e.get('avg_us', 0):8.2f} pct={e.get('time_pct', 0):5.1f} "
              f"MB={e.get('traffic_bytes_per_launch', 0) / 1e6:8.3f} GB/s={e.get('traffic_GBps', 0):7.0f} "
              f"mfmaTF={e.get('mfma_f64_TFLOPs') or 0:6.2f} busy={e.get('mfma_busy_frac') or 0:.4f}")


if __name__ == "__main__":
    main()
