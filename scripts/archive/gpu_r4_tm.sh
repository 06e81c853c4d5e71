#!/bin/bash
# Kernel tests (incl. the 1x1 GEMM 16-row-tile instances, the gather kernel's VALU
# remainder and the fuse adjoint's one-pass route), then knob A/B (conv_bench + step).
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_tm.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-tm}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest --maxfail=3 -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_heads_gpu.py tests/test_bench_instances_gpu.py \
  tests/test_lazy_bn_gpu.py -m gpu > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
CB_TUNES=${CB_TUNES:-"default 4=8,5=1 6=1"} AB_TUNES=${AB_TUNES:-"default 6=1 4=8,5=1"} \
  bash scripts/gpu_r4_knobs.sh ${TAG}
