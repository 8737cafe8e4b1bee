#!/bin/bash
# which device buffer holds a read-before-write: the parity tests with one
# buffer poisoned (NaN bytes) at a time (DYNOHIP_POISON_MASK bits, solver.cpp)
o=gpurun_out/${1:-pprobe}; mkdir -p $o
for b in 0 1 2 3 4 5 6 7 8 9 10; do
  DYNOHIP_POISON_MASK=$((1 << b)) timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 60 --timeout-method thread > $o/bit$b.log 2>&1
  echo "bit $b: $(tail -1 $o/bit$b.log)" >> $o/summary.txt
done
true
