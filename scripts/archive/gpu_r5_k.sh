#!/bin/bash
# SQ counters: dconv3_kernel (tune 9=0) vs dconv3s_kernel (9=1) on the 18-channel shape.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_sqpmc.sh sq5a_s3 3 dconv3 "--tune 9=0" && bash scripts/gpu_sqpmc.sh sq5b_s3 3 dconv3 "--tune 9=1" && \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5a > gpurun_out/sq5a_summary.txt 2>&1; \
python vae-2_amd/tools/sq_summary.py gpurun_out sq5b > gpurun_out/sq5b_summary.txt 2>&1; tail -40 gpurun_out/sq5b_summary.txt
