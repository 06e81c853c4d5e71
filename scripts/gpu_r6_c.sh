#!/bin/bash
# Probe: which fork/join pattern makes HIP graph capture_end crash (stop at the first failure)
set -o pipefail
mkdir -p gpurun_out
run() { timeout -k 10 120 python -u scripts/probe_lane_capture.py "$@" > gpurun_out/r6_c_$1_$2_$4_$5.log 2>&1; rc=$?; echo "$* rc=$rc"; tail -2 gpurun_out/r6_c_$1_$2_$4_$5.log; return $rc; }
run nest 3 100 3 0 && run nest 3 100 2 1
