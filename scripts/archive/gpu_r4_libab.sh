#!/bin/bash
# Training-step A/B of the in-tree build against vae-2_amd/vae2/ab/$2 (VAE2_LIB), interleaved.
#   gpurun --timeout 900 -- bash scripts/gpu_r4_libab.sh TAG OLD.so
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-lab}
OLD=$PWD/vae-2_amd/vae2/ab/${2:-old.so}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  ${TESTS:-tests/test_kernels_gpu.py tests/test_lazy_bn_gpu.py} -k "${TESTK:-bn or BatchNorm or lazy or resbn or fuse}" -m gpu \
  > gpurun_out/${TAG}_tests.log 2>&1 || { tail -20 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
i=0
for rep in 1 2 3; do
  for v in new old; do
    i=$((i+1))
    if [ $v = old ]; then
      VAE2_LIB=$OLD timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
        > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    else
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
        > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    fi
    echo "[$v] $(grep '^{' gpurun_out/${TAG}_ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
