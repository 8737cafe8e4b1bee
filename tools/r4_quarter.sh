#!/bin/bash
# Reduced gather, four lanes per entry for classes of <= 16 entries
# (DYNOHIP_GRED_QUARTER=1) against the default: bits and kernel stats.
set -o pipefail
o=gpurun_out/r4q
mkdir -p $o
timeout -k 10 300 python -u tools/ab_bits.py run $o/half.npz C1 C2 NS > $o/ab_half.log 2>&1 || exit 1
DYNOHIP_GRED_QUARTER=1 timeout -k 10 300 python -u tools/ab_bits.py run $o/quarter.npz C1 C2 NS > $o/ab_quarter.log 2>&1 || exit 2
python tools/ab_bits.py cmp $o/half.npz $o/quarter.npz > $o/ab_cmp.log 2>&1
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 3
DYNOHIP_GRED_QUARTER=1 bash tools/prof_run.sh $o/prof_ns_q bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns_q.txt 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 5
DYNOHIP_GRED_QUARTER=1 bash tools/prof_run.sh $o/prof_c2_q bench.py --steps 3 --no-cpu-baseline > $o/prof_c2_q.txt 2>&1 || exit 6
DYNOHIP_GRED_QUARTER=1 bash tools/prof_run.sh $o/prof_stream_q bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream_q.txt 2>&1 || exit 7
