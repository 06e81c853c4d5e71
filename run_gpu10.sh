#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() { local t=$1; shift; echo "== $*"; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi; }
step 300 python -m pytest tests/test_dist_gpu.py -x -q > gpurun_out/r10_dist.log 2>&1
tail -3 gpurun_out/r10_dist.log
step 700 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r10 -o run -- python bench.py > gpurun_out/r10_bench_prof.log 2>&1
grep '^{' gpurun_out/r10_bench_prof.log | cut -c1-120
step 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "igemm_kernel<4, 4, true, 0>" -f csv -d gpurun_out/pmc10_fetch -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r10_pmc1.log 2>&1
step 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "igemm_kernel<4, 4, true, 0>" -f csv -d gpurun_out/pmc10_write -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r10_pmc2.log 2>&1
step 400 python bench.py > gpurun_out/r10_bench.log 2>&1
grep '^{' gpurun_out/r10_bench.log
