#!/bin/bash
# Round 6: the multi-layer BatchNorm apply kernels striding over their pixel chunks in whole
# rounds (set_tune key 20 = resident-block budget) -- BN tests, bn_bench, step A/B (3 reps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_lazy_bn_gpu.py -k "bn or BN or multi or lazy" \
  > gpurun_out/r6_y_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6_y_tests.log; exit 1; }
tail -1 gpurun_out/r6_y_tests.log
for t in 0 1280 2560; do
  for set in narrow level wide; do
    timeout -k 10 120 python -u vae-2_amd/tools/bn_bench.py --set $set --res 0 --tune 20=$t > gpurun_out/r6_y_bn_${t}_$set.txt 2>&1 || { tail gpurun_out/r6_y_bn_${t}_$set.txt; exit 1; }
    echo "== key20=$t $set"; grep -v amdgpu.ids gpurun_out/r6_y_bn_${t}_$set.txt
  done
done
for rep in 1 2 3; do
  for t in none 20=1280 20=2560; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_y_${t}_${rep}.json 2> gpurun_out/r6_y_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_y_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_y_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
