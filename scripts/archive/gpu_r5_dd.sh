#!/bin/bash
# SQ counters of the 8-wave narrow weight gradient (default key 7 = 3) at 18 / 36 / 72 channels.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_sqpmc.sh sq5g_s3 3 wgrad3n && bash scripts/gpu_sqpmc.sh sq5g_s4 4 wgrad3n && \
bash scripts/gpu_sqpmc.sh sq5g_s5 5 wgrad3n && \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5g > gpurun_out/sq5g_summary.txt 2>&1; echo rc=$?
