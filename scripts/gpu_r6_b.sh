#!/bin/bash
# Round 6: level lanes (concurrent streams per HRNet depth level in the captured graph):
# graph == eager bit-identity, then an interleaved A/B of the default bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_graph_gpu.py > gpurun_out/r6_b_tests.log 2>&1 || { echo "graph tests failed"; tail -30 gpurun_out/r6_b_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r6_b_tests.log | tail -3
for rep in 1 2; do
  for ln in 0 4; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      --level-lanes $ln > gpurun_out/r6_b_lanes${ln}_${rep}.json 2> gpurun_out/r6_b_lanes${ln}_${rep}.err || { echo "bench lanes $ln failed"; tail -20 gpurun_out/r6_b_lanes${ln}_${rep}.err; exit 1; }
    python - <<PY
import json; d=json.loads(open("gpurun_out/r6_b_lanes${ln}_${rep}.json").read().strip().splitlines()[-1])
print("lanes ${ln} rep ${rep}:", d["value"], "frames/s", d["ms_per_step"], "ms/step")
PY
  done
done
