#!/bin/bash
# Round 6: the fuse sum + ReLU a channel quad per thread (set_tune key 21, on) -- fuse / lazy-BN
# / knob / bench-instance tests, step A/B against the per-channel form (3 reps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_lazy_bn_gpu.py tests/test_launch_knobs_gpu.py \
  tests/test_bench_instances_gpu.py tests/test_model_gpu.py \
  > gpurun_out/r6_bb_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_bb_tests.log | head -30; tail -5 gpurun_out/r6_bb_tests.log; exit 1; }
tail -1 gpurun_out/r6_bb_tests.log
for rep in 1 2 3; do
  for t in none 21=0; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_bb_${t}_${rep}.json 2> gpurun_out/r6_bb_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_bb_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_bb_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-pmc --profile-json gpurun_out/r6_bb_profile.json > gpurun_out/r6_bb_prof.log 2>&1 || exit 1
python -c "
import json; p=json.load(open('gpurun_out/r6_bb_profile.json'))
print([(f['name'], f['ms_per_step']) for f in p['families'] if f['name']=='fuse_resample'])
print([(k['name'], k['ms_per_step'], k['avg_us']) for k in p['kernels'] if 'fuse' in k['name']])"
