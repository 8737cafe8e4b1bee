#!/bin/bash
# Reduced gather: targets of > 32 entries on two waves (gather_band_wide);
# bits against the round's previous build (variants/old), kernel stats, bench
# lines, then the -m gpu suite and smoke().
set -o pipefail
o=gpurun_out/r4g5
mkdir -p $o
DYNOSAM_AMD_LIB_DIR=variants/old timeout -k 10 300 python -u tools/ab_bits.py run $o/old.npz C1 C2 NS > $o/ab_old.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/ab_bits.py run $o/new.npz C1 C2 NS > $o/ab_new.log 2>&1 || exit 2
python tools/ab_bits.py cmp $o/old.npz $o/new.npz > $o/ab_cmp.log 2>&1
bash tools/prof_run.sh $o/prof_ns bench.py --config NS --steps 2 --no-cpu-baseline > $o/prof_ns.txt 2>&1 || exit 3
bash tools/prof_run.sh $o/prof_c2 bench.py --steps 3 --no-cpu-baseline > $o/prof_c2.txt 2>&1 || exit 4
bash tools/prof_run.sh $o/prof_stream bench.py --mode stream --steps 1 --warmup 0 > $o/prof_stream.txt 2>&1 || exit 5
timeout -k 10 300 python -u bench.py --config NS --no-cpu-baseline > $o/bench_ns.log 2>&1 || exit 6
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $o/bench_c2.log 2>&1 || exit 7
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -x > $o/gpu_tests.log 2>&1 || exit 8
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $o/smoke.log 2>&1 || exit 9
