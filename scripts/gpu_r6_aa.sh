#!/bin/bash
# Round 6: the direct 3x3 K split in 4 shares (16-wave workgroups, set_tune key 15 = 2) vs 2
# shares (key 15 = 1, the default) -- form / knob tests, conv_bench, step A/B (3 reps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dconv_forms_gpu.py tests/test_launch_knobs_gpu.py tests/test_kernels_gpu.py -k "not igemm_ksplit" \
  > gpurun_out/r6_aa_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_aa_tests.log | head -30; tail -5 gpurun_out/r6_aa_tests.log; exit 1; }
tail -1 gpurun_out/r6_aa_tests.log
for t in 1 2; do
  timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 5 --iters 50 --tune 15=$t > gpurun_out/r6_aa_cb_$t.log 2>&1 || { tail -20 gpurun_out/r6_aa_cb_$t.log; exit 1; }
  echo "conv_bench key15=$t"; tail -3 gpurun_out/r6_aa_cb_$t.log
done
for rep in 1 2 3; do
  for t in none 15=2; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_aa_${t}_${rep}.json 2> gpurun_out/r6_aa_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_aa_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_aa_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
