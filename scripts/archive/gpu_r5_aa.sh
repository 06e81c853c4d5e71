#!/bin/bash
# Narrow weight gradient with 8-wave workgroups (key 7 = 3) vs 4 (7 = 1): tests, conv_bench, step A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_wgrad_narrow_gpu.py \
  > gpurun_out/r5aa_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5aa_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/r5aa_tests.log | head -20; exit $rc; }
for t in 7=1 7=3 7=1 7=3; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 30 --tune $t \
    > gpurun_out/r5aa_$t.log 2>&1 || { tail -5 gpurun_out/r5aa_$t.log; exit 1; }
  echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5aa_$t.log
done
for t in 7=1 7=3 7=1 7=3; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5aa_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5aa_bench_$t.log; exit 1; }
  echo "[bench $t] $(grep '^{' gpurun_out/r5aa_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
