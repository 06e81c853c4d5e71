#!/bin/bash
# Round 6: level-lane variants A/B (0 = one stream, 2 / 4 lanes, -4 = forward only)
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for ln in 0 2 -4 -2; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      --level-lanes $ln > gpurun_out/r6_d_lanes${ln}_${rep}.json 2> gpurun_out/r6_d_lanes${ln}_${rep}.err || { echo "bench lanes $ln failed"; tail -20 gpurun_out/r6_d_lanes${ln}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_d_lanes${ln}_${rep}.json').read().strip().splitlines()[-1]); print('lanes ${ln} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
