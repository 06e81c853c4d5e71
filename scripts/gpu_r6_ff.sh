#!/bin/bash
# Round 6: SQ PMC before / after of the launch-shape changes on the narrow 3x3 convs --
# 72 -> 72 direct 3x3 without / with the K split (set_tune key 15 = 0 / 1) and 36 -> 36
# streaming 3x3 with two-step / one-step bands (key 17 = 2 / 1); three counter passes each
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_sqpmc.sh r6_ff_k15_0 5 dconv3_kernel "--tune 15=0" || exit 1
bash scripts/gpu_sqpmc.sh r6_ff_k15_1 5 dconv3_kernel "--tune 15=1" || exit 1
bash scripts/gpu_sqpmc.sh r6_ff_k17_2 4 dconv3s_kernel "--tune 17=2" || exit 1
bash scripts/gpu_sqpmc.sh r6_ff_k17_1 4 dconv3s_kernel "--tune 17=1" || exit 1
