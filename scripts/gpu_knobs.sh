#!/bin/bash
# bench.py under several environment settings in turn, baseline first and last.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for cfg in "BASE=1" "VAE2_DC_TM_TH=1536" "VAE2_DC_TM_TH=384" "VAE2_G1_PERCU=2" "VAE2_G1_PERCU=4" \
           "VAE2_KS_TH=1024" "VAE2_KS_TH=256" "VAE2_W3_RES=1024" "BASE=1"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
    > gpurun_out/knob_$i.log 2>&1 || { tail -20 gpurun_out/knob_$i.log; exit 1; }
  echo "[$cfg] $(grep '^{' gpurun_out/knob_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
