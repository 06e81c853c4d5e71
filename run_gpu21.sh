#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 300 python -m pytest tests/test_kernels_gpu.py -x -q -k "direct or conv" > gpurun_out/r21_kt.log 2>&1
tail -2 gpurun_out/r21_kt.log
grep -q " passed" gpurun_out/r21_kt.log && ! grep -q "failed" gpurun_out/r21_kt.log || exit 1
step 300 python vae-2_amd/tools/conv_bench.py --algo 0 --only 1 2 8 > gpurun_out/r21_conv.log 2>&1
cat gpurun_out/r21_conv.log | grep -v amdgpu.ids
