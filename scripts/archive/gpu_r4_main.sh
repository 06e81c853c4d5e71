#!/bin/bash
# Round-4 main GPU call: the distributed-step probe (eager, bounded), the -m gpu suite,
# then the default bench line.
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_main.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-m4}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 150 python -u vae-2_amd/tools/dist_step_probe.py --steps 3 \
  > gpurun_out/${TAG}_probe.log 2>&1; rc=$?
cat gpurun_out/${TAG}_probe.log | grep -v amdgpu.ids
[ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
timeout -k 10 900 python -u -m pytest --maxfail=4 -v --timeout 420 --timeout-method thread \
  tests -m gpu > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench.log | cut -c1-900
