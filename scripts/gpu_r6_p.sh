#!/bin/bash
# Round 6: the grouped-launch test with key 15 pinned off, then launch-shape A/B in the step:
# default, key 2 = 1 (direct 3x3 8-row tiles as 8 one-row waves), key 0 = 512 / 1024 (gather
# GEMM row tiles shrink until the grid reaches that many workgroups)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "grouped" > gpurun_out/r6_p_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6_p_tests.log; exit 1; }
tail -1 gpurun_out/r6_p_tests.log
for rep in 1 2; do
  for t in none 2=1 0=512 0=1024; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_p_${t}_${rep}.json 2> gpurun_out/r6_p_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_p_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_p_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
