#!/bin/bash
# Round 6: the full -m gpu suite with the K-split direct 3x3 on by default, then 2 more step
# A/B pairs of set_tune key 15
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/r6_o_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r6_o_tests.log | head -30; tail -5 gpurun_out/r6_o_tests.log; exit 1; }
tail -2 gpurun_out/r6_o_tests.log
for rep in 1 2; do
  for t in 0 1; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline --conv-tune 15=$t \
      > gpurun_out/r6_o_${t}_${rep}.json 2> gpurun_out/r6_o_${t}_${rep}.err || { echo "bench $t failed"; tail -20 gpurun_out/r6_o_${t}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_o_${t}_${rep}.json').read().strip().splitlines()[-1]); print('key15=${t} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
