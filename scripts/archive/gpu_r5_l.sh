#!/bin/bash
# Round 5: streaming direct 3x3 for the 18 / 36-channel branches (tune key 9): its tests,
# the kernel suites that route through it, conv microbench A/B, step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dconv_stream_gpu.py \
  > gpurun_out/r5l_stream.log 2>&1
rc=$?; echo "stream tests rc=$rc"; tail -3 gpurun_out/r5l_stream.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5l_stream.log | head -30; exit $rc; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_lazy_bn_gpu.py tests/test_model_gpu.py tests/test_dist_gpu.py -s > gpurun_out/r5l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5l_tests.log; grep -E "W18 2 ranks" gpurun_out/r5l_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5l_tests.log | head -20; exit $rc; }
for t in 9=0 9=1 9=2; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 20 --tune $t \
    > gpurun_out/r5l_conv_$t.log 2>&1 || { tail -5 gpurun_out/r5l_conv_$t.log; exit 1; }
  echo "== conv tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5l_conv_$t.log
done
for t in 9=0 9=1 9=0 9=1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5l_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5l_bench_$t.log; exit 1; }
  echo "[bench tune $t] $(grep '^{' gpurun_out/r5l_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
