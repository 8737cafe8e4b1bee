#!/bin/bash
# A/B of the try-result wait (event polling vs hipEventSynchronize) on the
# sliding-window stream and C2, each run under its own limit.
set -o pipefail
mkdir -p gpurun_out
for w in spin block spin block; do
  DYNOHIP_RESULT_WAIT=$w timeout -k 10 200 python -u bench.py --mode stream --steps 3 --warmup 1 > gpurun_out/ab_stream_$w.log 2>&1 || exit 1
  grep '^{' gpurun_out/ab_stream_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('stream', '$w', round(d['value'],1), round(d['ms_per_solve_incl_upload'],3), round(d['ms_per_frame_construction'],3))" >> gpurun_out/ab_wait.txt
  DYNOHIP_RESULT_WAIT=$w timeout -k 10 200 python -u bench.py --steps 20 --no-cpu-baseline > gpurun_out/ab_c2_$w.log 2>&1 || exit 2
  grep '^{' gpurun_out/ab_c2_$w.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C2', '$w', round(d['value'],1), d.get('ms_full_batch_opt'))" >> gpurun_out/ab_wait.txt
done
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_backend.py -m gpu > gpurun_out/ab_tests.log 2>&1 || exit 3
