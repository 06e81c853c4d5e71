#!/bin/bash
# Round-6 evidence in one call: the full -m gpu suite, the default bench line (CPU baseline,
# live PMC traffic + rocprofv3 trace average of the dominant kernel), the profiled bench +
# rocprofv3 kernel trace / stats + step breakdown, the bf16-operand and 256x512 lines.
#   gpurun --timeout 1200 -- bash scripts/gpu_r6_final.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-r6f}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench_default.log 2>&1 \
  || { tail -20 gpurun_out/${TAG}_bench_default.log; exit 1; }
grep '^{' gpurun_out/${TAG}_bench_default.log | cut -c1-300
bash scripts/gpu_bench_prof.sh $TAG || exit 1
for v in "bf16::--dtype bf16" "256x512::--height 256 --width 512 --batch 2" \
         "bf16_256x512::--dtype bf16 --height 256 --width 512 --batch 2"; do
  name=${v%%::*}; args=${v#*::}
  timeout -k 10 400 python bench.py --no-cpu-baseline $args \
    --profile-json gpurun_out/${TAG}_profile_${name}.json > gpurun_out/${TAG}_bench_${name}.log 2>&1 \
    || { tail -20 gpurun_out/${TAG}_bench_${name}.log; exit 1; }
  grep '^{' gpurun_out/${TAG}_bench_${name}.log | cut -c1-200
done
