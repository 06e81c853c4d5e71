#!/bin/bash
# Stride-2 18->36 conv (gather kernel): conv_bench timing + SQ counters (igemm / wgrad).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 9 --iters 20 > gpurun_out/r5s_conv.log 2>&1 || { tail -5 gpurun_out/r5s_conv.log; exit 1; }
grep -E "^[0-9]+x[0-9]+" gpurun_out/r5s_conv.log
bash scripts/gpu_sqpmc.sh sq5f_s9 9 "igemm|wgrad_kernel" && \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5f > gpurun_out/sq5f_summary.txt 2>&1; echo rc=$?
