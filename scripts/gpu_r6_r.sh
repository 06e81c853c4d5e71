#!/bin/bash
# Round 6: the full -m gpu suite with key 15 (K-split direct 3x3) and key 0 = 512 (gather
# GEMM minimum workgroups) on by default, then step A/B of key 16 = 1 (narrow weight
# gradient: one tile per split) and key 17 = 1 (streaming 3x3: one step per band)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/r6_r_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r6_r_tests.log | head -30; tail -5 gpurun_out/r6_r_tests.log; exit 1; }
tail -1 gpurun_out/r6_r_tests.log
for rep in 1 2; do
  for t in none 16=1 17=1; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_r_${t}_${rep}.json 2> gpurun_out/r6_r_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_r_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_r_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
