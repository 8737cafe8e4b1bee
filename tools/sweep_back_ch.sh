set -o pipefail
o=gpurun_out/swch; mkdir -p $o
DYNOSAM_AMD_LIB_DIR=build_ch4 DYNOHIP_BACK_PART_TILES=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $o/parity.log 2>&1 || exit 1
for cfg in C2 NS; do
  timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu-baseline > $o/base_$cfg.log 2>&1 || exit 2
  for t in 2 4; do DYNOSAM_AMD_LIB_DIR=build_ch4 DYNOHIP_BACK_PART_TILES=$t timeout -k 10 200 python -u bench.py --config $cfg --steps 10 --no-cpu-baseline > $o/ch4_t${t}_$cfg.log 2>&1 || exit 3; done
done
