#!/bin/bash
# Streaming 36-channel conv on by default: tests, step A/B (tune 9 = 0 / 2 / 3).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dconv_stream_gpu.py \
  tests/test_kernels_gpu.py tests/test_lazy_bn_gpu.py tests/test_model_gpu.py -s > gpurun_out/r5o_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5o_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5o_tests.log | head -20; exit $rc; }
for t in 9=0 9=2 9=3 9=0 9=2 9=3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5o_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5o_bench_$t.log; exit 1; }
  echo "[bench tune $t] $(grep '^{' gpurun_out/r5o_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
