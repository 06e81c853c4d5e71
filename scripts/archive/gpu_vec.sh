#!/bin/bash
# conv kernels with / without the quad-transposed 16-byte epilogue stores (set_algo bit 64),
# tests, bench
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu \
  -k "${1:-gemm1x1 or conv_fwd_bwd or direct_conv3x3 or conv_bn or lazy or ksplit}" > gpurun_out/vec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/vec_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/vec_tests.log | head -20; exit $rc; }
timeout -k 10 300 python vae-2_amd/tools/conv_bench.py --all --iters 20 --algo 0 64 > gpurun_out/vec_cb.log 2>&1 \
  || { tail gpurun_out/vec_cb.log; exit 1; }
grep -E "algo|weighted" gpurun_out/vec_cb.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/vec_bench.log 2>&1 \
  || { tail -20 gpurun_out/vec_bench.log; exit 1; }
grep '^{' gpurun_out/vec_bench.log | cut -c1-200
