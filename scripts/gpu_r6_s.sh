#!/bin/bash
# Round 6: streaming 3x3 band sizing in the step -- key 17 = 1 (one 4-row step per band
# allowed: the 36-channel layers get 512 instead of 256 workgroups), and with key 10 = 8
# (18 channels: target 8 workgroups per CU, one step per band), 3 interleaved reps
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in none 17=1 17=1,10=8; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_s_${t}_${rep}.json 2> gpurun_out/r6_s_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_s_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_s_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
for t in 0 1; do
  timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 3 4 --iters 50 --tune 17=$t > gpurun_out/r6_s_cb_$t.log 2>&1 || { tail -20 gpurun_out/r6_s_cb_$t.log; exit 1; }
  echo "conv_bench key17=$t"; tail -5 gpurun_out/r6_s_cb_$t.log
done
