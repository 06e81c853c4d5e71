#!/bin/bash
# conv microbenchmark at several batch sizes (per-launch fixed cost vs work)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 8 16 32; do
  timeout -k 10 200 python vae-2_amd/tools/conv_bench.py --only 0 2 3 4 5 6 8 9 --iters 20 --batch $b \
    > gpurun_out/scal_$b.log 2>&1 || { tail gpurun_out/scal_$b.log; exit 1; }
  echo "== batch $b"; grep -E "^[0-9]+x" gpurun_out/scal_$b.log
done
