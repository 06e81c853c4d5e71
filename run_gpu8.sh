#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
K='igemm_kernel<4, 4, true, 0>'
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_r8 -o run -- python bench.py > gpurun_out/r8_bench_prof.log 2>&1 || exit $?
echo prof-ok
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "igemm_kernel<4, 4, true, 0>" -f csv -d gpurun_out/pmc_fetch -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r8_pmc1.log 2>&1 || exit $?
echo pmc1-ok
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "igemm_kernel<4, 4, true, 0>" -f csv -d gpurun_out/pmc_write -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-roofline > gpurun_out/r8_pmc2.log 2>&1 || exit $?
echo pmc2-ok
timeout -k 10 400 python bench.py > gpurun_out/r8_bench.log 2>&1
grep '^{' gpurun_out/r8_bench.log
