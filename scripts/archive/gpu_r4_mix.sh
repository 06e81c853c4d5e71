#!/bin/bash
# Test + measure round: heads / kernel / bench-instance tests, head_bench, conv_bench over
# every ELBO shape, then the training step (default, and with heads algo ${ALT:-8}).
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_mix.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-mx}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail=3 -q --timeout 300 --timeout-method thread \
  tests/test_heads_gpu.py tests/test_kernels_gpu.py tests/test_bench_instances_gpu.py \
  tests/test_lazy_bn_gpu.py -m gpu \
  > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
timeout -k 10 120 python vae-2_amd/tools/head_bench.py > gpurun_out/${TAG}_hb.log 2>&1 || { tail -5 gpurun_out/${TAG}_hb.log; exit 1; }
cat gpurun_out/${TAG}_hb.log
timeout -k 10 180 python vae-2_amd/tools/conv_bench.py --all --iters 20 > gpurun_out/${TAG}_cb.log 2>&1 || { tail -5 gpurun_out/${TAG}_cb.log; exit 1; }
grep weighted gpurun_out/${TAG}_cb.log
i=0
for v in 0 ${ALT:-8} 0; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 --heads-algo $v \
    > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
  echo "[$v] $(grep '^{' gpurun_out/${TAG}_ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
