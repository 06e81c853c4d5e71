#!/bin/bash
# Round 6: the full -m gpu suite with key 15 (K-split direct 3x3) and key 0 = 512 (gather
# GEMM minimum workgroups) on by default, then the default bench line
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/r6_r_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r6_r_tests.log | head -30; tail -5 gpurun_out/r6_r_tests.log; exit 1; }
tail -1 gpurun_out/r6_r_tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline > gpurun_out/r6_r_bench.json 2> gpurun_out/r6_r_bench.err || { tail -20 gpurun_out/r6_r_bench.err; exit 1; }
tail -1 gpurun_out/r6_r_bench.json | cut -c1-220
