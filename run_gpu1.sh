#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/r1_kernels.log 2>&1
tail -5 gpurun_out/r1_kernels.log
step 600 python -m pytest tests/test_model_gpu.py -q > gpurun_out/r1_model.log 2>&1
tail -5 gpurun_out/r1_model.log
step 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1
tail -3 gpurun_out/r1_smoke.log
step 400 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r1_bench.log 2>&1
tail -3 gpurun_out/r1_bench.log
