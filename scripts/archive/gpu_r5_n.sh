#!/bin/bash
# SQ counters of the streaming kernel (18 ch: global weights, 4 workgroups per CU target;
# 36 ch) and dconv3_kernel on the 36-channel shape.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_sqpmc.sh sq5c_s3 3 dconv3 "--tune 9=2,11=0,10=4" && \
bash scripts/gpu_sqpmc.sh sq5c_s4 4 dconv3 "--tune 9=2,11=0,10=4" && \
bash scripts/gpu_sqpmc.sh sq5d_s4 4 dconv3 "--tune 9=0" && \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5c > gpurun_out/sq5c_summary.txt 2>&1 && \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5d > gpurun_out/sq5d_summary.txt 2>&1; echo rc=$?
