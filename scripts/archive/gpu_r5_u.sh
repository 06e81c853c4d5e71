#!/bin/bash
# Gather GEMM with the K-step table: conv tests, stride-2 / all shapes microbench, step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_bench_instances_gpu.py tests/test_lazy_bn_gpu.py tests/test_kernels_gpu.py \
  tests/test_model_gpu.py > gpurun_out/r5u_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5u_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5u_tests.log | head -20; exit $rc; }
for t in 12=0 12=1; do
timeout -k 10 200 python vae-2_amd/tools/conv_bench.py --all --iters 20 --tune $t > gpurun_out/r5u_conv_$t.log 2>&1 || { tail -5 gpurun_out/r5u_conv_$t.log; exit 1; }
echo "== conv tune $t"; grep -E "^[0-9]+x[0-9]+|total" gpurun_out/r5u_conv_$t.log
done
for t in 12=0 12=1 12=0 12=1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5u_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5u_bench_$t.log; exit 1; }
  echo "[bench $t] $(grep '^{' gpurun_out/r5u_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
