mkdir -p gpurun_out/t1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_partition.py -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/t1/tests.log 2>&1; echo tests_rc=$? >> gpurun_out/t1/tests.log
DYNOSAM_AMD_LIB_DIR=variants/tclk timeout -k 10 150 python -u tools/task_clock.py C2 gpurun_out/t1/c2.json > gpurun_out/t1/c2.txt 2>&1 || exit 2
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/t1/bench.log 2>&1 || exit 3
