#!/bin/bash
# Round 6: the direct 3x3 K split over 8 waves for layers short of workgroups (set_tune
# key 15) -- parity tests of both forms, isolated conv timing, step A/B pairs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dconv_forms_gpu.py \
  > gpurun_out/r6_n_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_n_tests.log | head -30; tail -5 gpurun_out/r6_n_tests.log; exit 1; }
tail -2 gpurun_out/r6_n_tests.log
for t in 0 1; do
  timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 5 --iters 50 --tune 15=$t > gpurun_out/r6_n_cb_$t.log 2>&1 || { tail -20 gpurun_out/r6_n_cb_$t.log; exit 1; }
  echo "conv_bench key15=$t"; tail -4 gpurun_out/r6_n_cb_$t.log
done
for rep in 1 2; do
  for t in 1 0; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --conv-tune 15=$t \
      > gpurun_out/r6_n_${t}_${rep}.json 2> gpurun_out/r6_n_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_n_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_n_${t}_${rep}.json').read().strip().splitlines()[-1]); print('key15=${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
