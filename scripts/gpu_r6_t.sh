#!/bin/bash
# Round 6: streaming 3x3 one-step bands by default (key 17 = 1) -- the conv suites, then
# step A/B against key 17 = 2 (3 interleaved reps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dconv_stream_gpu.py tests/test_dconv_forms_gpu.py tests/test_bench_instances_gpu.py \
  tests/test_model_gpu.py tests/test_lazy_bn_gpu.py tests/test_partbn_gpu.py \
  > gpurun_out/r6_t_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_t_tests.log | head -30; tail -5 gpurun_out/r6_t_tests.log; exit 1; }
tail -1 gpurun_out/r6_t_tests.log
for rep in 1 2 3; do
  for t in none 17=2; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_t_${t}_${rep}.json 2> gpurun_out/r6_t_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_t_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_t_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
for t in 1 2; do
  timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 3 4 --iters 50 --tune 17=$t > gpurun_out/r6_t_cb_$t.log 2>&1 || { tail -20 gpurun_out/r6_t_cb_$t.log; exit 1; }
  echo "conv_bench key17=$t"; tail -5 gpurun_out/r6_t_cb_$t.log
done
