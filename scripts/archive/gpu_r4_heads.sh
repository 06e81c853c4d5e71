#!/bin/bash
# Head-kernel round: the head / adjoint tests, head_bench, then the training step with the
# one-pass adjoint (default) and the two-pass form (heads algo 4), twice interleaved.
#   gpurun --timeout 900 -- bash scripts/gpu_r4_heads.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-hd}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_heads_gpu.py -m gpu > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
timeout -k 10 120 python vae-2_amd/tools/head_bench.py > gpurun_out/${TAG}_hb.log 2>&1 || { tail -5 gpurun_out/${TAG}_hb.log; exit 1; }
cat gpurun_out/${TAG}_hb.log
i=0
for rep in 1 2; do
  for v in 0 ${ALT:-4}; do
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 --heads-algo $v \
      > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    echo "[$v] $(grep '^{' gpurun_out/${TAG}_ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
