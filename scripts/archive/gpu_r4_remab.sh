#!/bin/bash
# New build vs the previous one (vae-2_amd/vae2/ab/libvae2_hip_r4a.so, run with the same
# launch knobs): the -m gpu suite on the new build, conv_bench over every ELBO shape on
# both, then the training step on both, twice interleaved.
#   gpurun --timeout 1200 -- bash scripts/gpu_r4_remab.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-ra}
OLD=$PWD/vae-2_amd/vae2/ab/libvae2_hip_r4a.so
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest --maxfail=3 -q --timeout 300 --timeout-method thread \
  tests -m gpu -k "bench_instances or kernels or lazy_bn or model" > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" gpurun_out/${TAG}_tests.log | head -30; exit $rc; }
timeout -k 10 180 python vae-2_amd/tools/conv_bench.py --all --iters 20 > gpurun_out/${TAG}_cb_new.log 2>&1 || exit 1
VAE2_LIB=$OLD timeout -k 10 180 python vae-2_amd/tools/conv_bench.py --all --iters 20 --tune 1=1,3=1 \
  > gpurun_out/${TAG}_cb_old.log 2>&1 || exit 1
echo "new: $(grep weighted gpurun_out/${TAG}_cb_new.log)"
echo "old: $(grep weighted gpurun_out/${TAG}_cb_old.log)"
i=0
for rep in 1 2; do
  for v in new old; do
    i=$((i+1))
    if [ $v = old ]; then
      VAE2_LIB=$OLD timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
        --conv-tune 1=1,3=1 > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    else
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --steps 20 \
        > gpurun_out/${TAG}_ab_$i.log 2>&1 || { tail -5 gpurun_out/${TAG}_ab_$i.log; exit 1; }
    fi
    echo "[$v] $(grep '^{' gpurun_out/${TAG}_ab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  done
done
