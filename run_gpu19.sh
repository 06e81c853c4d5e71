#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 600 python -m pytest tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_dist_gpu.py -x -q > gpurun_out/r19_mt.log 2>&1
tail -3 gpurun_out/r19_mt.log
step 600 rocprofv3 --kernel-trace -f csv -d gpurun_out/prof_r19 -o run -- python bench.py --no-cpu-baseline --no-roofline --steps 10 --warmup 2 > gpurun_out/r19_prof.log 2>&1
python vae-2_amd/tools/trace_steps.py gpurun_out/prof_r19/run_kernel_trace.csv > gpurun_out/r19_steps.txt 2>&1
head -30 gpurun_out/r19_steps.txt
