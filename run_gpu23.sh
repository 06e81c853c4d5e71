#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/r23_kt.log 2>&1
tail -3 gpurun_out/r23_kt.log
grep -q " passed" gpurun_out/r23_kt.log && ! grep -q "failed" gpurun_out/r23_kt.log || exit 1
step 300 python vae-2_amd/tools/conv_bench.py --algo 0 > gpurun_out/r23_conv.log 2>&1
cat gpurun_out/r23_conv.log | grep -v amdgpu.ids
step 600 python -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py -x -q > gpurun_out/r23_mt.log 2>&1
tail -3 gpurun_out/r23_mt.log
step 400 python bench.py --no-cpu-baseline > gpurun_out/r23_bench.log 2>&1
grep '^{' gpurun_out/r23_bench.log | cut -c1-300
