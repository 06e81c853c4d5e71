#!/bin/bash
# Round 6: BN partials from the gather / 1x1 GEMM data-gradient epilogues (ops.PartBN) --
# kernel + block tests, the suites that touch the changed paths, step A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_partbn_gpu.py tests/test_lazy_bn_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py \
  tests/test_bench_instances_gpu.py tests/test_dist_gpu.py tests/test_kernels_gpu.py \
  > gpurun_out/r6_j_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_j_tests.log | head -30; tail -5 gpurun_out/r6_j_tests.log; exit 1; }
tail -2 gpurun_out/r6_j_tests.log
for rep in 1 2; do
  for pb in on off; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --part-bn $pb \
      > gpurun_out/r6_j_${pb}_${rep}.json 2> gpurun_out/r6_j_${pb}_${rep}.err || { echo "bench $pb failed"; tail -20 gpurun_out/r6_j_${pb}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_j_${pb}_${rep}.json').read().strip().splitlines()[-1]); print('part-bn ${pb} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
