#!/bin/bash
# SQ counters of the narrow 3x3 weight gradient (wgrad3n) at 18 / 36 / 72 channels.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_sqpmc.sh sq5e_s3 3 wgrad3n && bash scripts/gpu_sqpmc.sh sq5e_s4 4 wgrad3n && \
bash scripts/gpu_sqpmc.sh sq5e_s5 5 wgrad3n && \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5e > gpurun_out/sq5e_summary.txt 2>&1; echo rc=$?
