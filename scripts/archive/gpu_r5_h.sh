#!/bin/bash
# Round 5: BN backward reduce specialised too: tests, microbench, step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_lazy_bn_gpu.py tests/test_model_gpu.py tests/test_dist_gpu.py tests/test_syncbn_ipc_gpu.py -s \
  > gpurun_out/r5h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5h_tests.log; grep -E "exchange|W18 2 ranks" gpurun_out/r5h_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5h_tests.log | head -20; exit $rc; }
for t in 8=1; do
  for m in 0 1; do
    timeout -k 10 120 python vae-2_amd/tools/bn_bench.py --tune $t --mask $m > gpurun_out/r5h_bn_${t}_${m}.log 2>&1 || { tail -5 gpurun_out/r5h_bn_${t}_${m}.log; exit 1; }
    echo "== bn tune $t mask $m"; grep -v amdgpu.ids gpurun_out/r5h_bn_${t}_${m}.log
  done
done
for t in 8=1 8=1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5h_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5h_bench_$t.log; exit 1; }
  echo "[bench tune $t] $(grep '^{' gpurun_out/r5h_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
