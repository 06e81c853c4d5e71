#!/bin/bash
# Launch-shape knob A/B: per-kernel times over every ELBO conv shape (conv_bench), then
# the training step itself (bench.py, 20 steps, graph replay) per knob, twice interleaved.
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_knobs.sh TAG   (CB_TUNES / AB_TUNES: the
#   knob settings to time, space-separated, "default" for none)
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-k4}
mkdir -p gpurun_out
export TMPDIR=/tmp
CB_TUNES=${CB_TUNES:-"default 2=1 3=1 0=1024 1=1"}
AB_TUNES=${AB_TUNES:-"default 2=1 3=1 0=1024 1=1 0=1024,1=1,2=1,3=1"}
for tune in $CB_TUNES; do
  [ "$tune" = default ] && tune=""
  timeout -k 10 180 python vae-2_amd/tools/conv_bench.py --all --iters 20 ${tune:+--tune $tune} \
    > gpurun_out/${TAG}_cb_${tune:-default}.log 2>&1 || { tail -5 gpurun_out/${TAG}_cb_${tune:-default}.log; exit 1; }
  echo "== conv_bench tune '${tune}': $(grep weighted gpurun_out/${TAG}_cb_${tune:-default}.log)"
done
i=0
for rep in 1 2; do
  for tune in $AB_TUNES; do
    [ "$tune" = default ] && tune=""
    i=$((i+1))
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
      ${tune:+--conv-tune $tune} > gpurun_out/${TAG}_ab_$i.log 2>&1 \
      || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    echo "[${tune:-default}] $(grep '^{' gpurun_out/${TAG}_ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
