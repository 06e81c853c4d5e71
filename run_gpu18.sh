#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 300 python tests/diag_grad_spread.py > gpurun_out/r18_diag.log 2>&1
cat gpurun_out/r18_diag.log | grep -v amdgpu.ids
step 300 python vae-2_amd/tools/conv_bench.py --algo 0 --only 3 4 5 6 > gpurun_out/r18_conv.log 2>&1
cat gpurun_out/r18_conv.log | grep -v amdgpu.ids
step 400 python bench.py --no-cpu-baseline > gpurun_out/r18_bench.log 2>&1
grep '^{' gpurun_out/r18_bench.log | cut -c1-300
