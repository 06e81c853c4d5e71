#!/bin/bash
# LazyBN tests + selected GPU tests, then bench A/B (lazy on / off).
#   gpurun -- bash scripts/gpu_lazy.sh "lazy or multi_bn or model"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
K=${1:-lazy}
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu \
  -k "$K" > gpurun_out/lazy_tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/lazy_tests.log | tail -40
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/lazy_tests.log | head -30; exit $rc; }
for ab in on off on; do
  timeout -k 10 400 python bench.py --no-cpu-baseline --no-roofline --lazy-bn $ab \
    > gpurun_out/lazy_bench_$ab.log 2>&1 || { tail -20 gpurun_out/lazy_bench_$ab.log; exit 1; }
  echo "lazy $ab: $(grep '^{' gpurun_out/lazy_bench_$ab.log | cut -c1-200)"
done
