#!/bin/bash
# Round 6: branch-free head output-stage passes -- tests, head microbench, step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_heads_gpu.py \
  > gpurun_out/r6_f_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6_f_tests.log; exit 1; }
tail -2 gpurun_out/r6_f_tests.log
timeout -k 10 120 python -u vae-2_amd/tools/head_bench.py --only out > gpurun_out/r6_f_headbench.txt 2>&1 || { tail gpurun_out/r6_f_headbench.txt; exit 1; }
cat gpurun_out/r6_f_headbench.txt | tail -14
for rep in 1 2; do
  for ha in 0 65536; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --heads-algo $ha \
      > gpurun_out/r6_f_${ha}_${rep}.json 2> gpurun_out/r6_f_${ha}_${rep}.err || { echo "bench $ha failed"; tail -20 gpurun_out/r6_f_${ha}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_f_${ha}_${rep}.json').read().strip().splitlines()[-1]); print('heads algo ${ha} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
