#!/bin/bash
# Round 6: launch sizing A/B in the step -- gather weight-gradient target workgroups (key 18)
# and BatchNorm blocks per layer (key 19), 2 interleaved reps
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for t in none 18=2048 19=2048 19=512; do
    if [ $t = none ]; then A=""; else A="--conv-tune $t"; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline $A \
      > gpurun_out/r6_u_${t}_${rep}.json 2> gpurun_out/r6_u_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_u_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_u_${t}_${rep}.json').read().strip().splitlines()[-1]); print('tune ${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
