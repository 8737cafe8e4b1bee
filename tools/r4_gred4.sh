#!/bin/bash
# Reduced gather: 16-byte operand row loads, two lanes per entry for classes
# of <= 32 entries (DYNOHIP_GRED_HALF=0: one lane); bits against the round's
# previous build (variants/old); kernel stats of NS, C2 and the stream.
set -o pipefail
o=gpurun_out/r4g4
mkdir -p $o
DYNOSAM_AMD_LIB_DIR=variants/old timeout -k 10 300 python -u tools/ab_bits.py run $o/old.npz C1 C2 NS > $o/ab_old.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bits.py run $o/new.npz C1 C2 NS > $o/ab_new.log 2>&1 || exit 2
python tools/ab_bits.py cmp $o/old.npz $o/new.npz > $o/ab_cmp.log 2>&1
DYNOHIP_GRED_HALF=0 timeout -k 10 300 python -u tools/ab_bits.py run $o/one.npz C1 C2 NS > $o/ab_one.log 2>&1 || exit 3
python tools/ab_bits.py cmp $o/old.npz $o/one.npz > $o/ab_cmp_one.log 2>&1
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 4
DYNOHIP_GRED_HALF=0 bash tools/prof_run.sh $o/prof_ns_one bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns_one.txt 2>&1 || exit 5
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 6
DYNOHIP_GRED_HALF=0 bash tools/prof_run.sh $o/prof_c2_one bench.py --steps 3 --no-cpu-baseline > $o/prof_c2_one.txt 2>&1 || exit 7
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 8
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 9
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit 10
