#!/bin/bash
# Round 6: every ELBO conv shape under the auto kernel choice vs gather-only vs direct-where-legal
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u vae-2_amd/tools/conv_bench.py --all --algo 0 1 2 --iters 20 \
  > gpurun_out/r6_i_convbench.txt 2>&1 || { tail -20 gpurun_out/r6_i_convbench.txt; exit 1; }
grep -E "^== |weighted" gpurun_out/r6_i_convbench.txt
