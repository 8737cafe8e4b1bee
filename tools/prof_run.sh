#!/bin/bash
# usage: tools/prof_run.sh <outdir> <python args...>  -- kernel-trace stats of one run
out=$1; shift
mkdir -p $out && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out -o run --output-format csv -- python "$@" > $out/stdout.log 2>&1
rc=$?
python - "$out" <<'PY'
import csv, sys, glob
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True) or glob.glob(sys.argv[1] + "/run_kernel_stats.csv")
rows = list(csv.DictReader(open(f[0])))
for r in rows[:14]:
    print(f"{r['Name'][:58]:58s} calls={r['Calls']:>6} total_ms={float(r['TotalDurationNs'])/1e6:9.3f} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
PY
exit $rc
