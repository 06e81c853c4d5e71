#!/bin/bash
# Round 6: narrow 3x3 weight gradient with bank-conflict-free halo rows (LDS row stride =
# CSW mod 16) -- parity tests, conv_bench wgrad + step A/B against the unpadded layout
# (libvae2_hip_base.so, built from the previous commit's wgrad_narrow.hip)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_wgrad_narrow_gpu.py tests/test_bench_instances_gpu.py \
  > gpurun_out/r6_l_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_l_tests.log | head -30; tail -5 gpurun_out/r6_l_tests.log; exit 1; }
tail -2 gpurun_out/r6_l_tests.log
for lib in new base; do
  if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
  VAE2_LIB=$PWD/$L timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 50 > gpurun_out/r6_l_cb_$lib.log 2>&1 || { tail -20 gpurun_out/r6_l_cb_$lib.log; exit 1; }
  echo "== conv_bench $lib"; tail -6 gpurun_out/r6_l_cb_$lib.log
done
for rep in 1 2; do
  for lib in new base; do
    if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
    VAE2_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      > gpurun_out/r6_l_${lib}_${rep}.json 2> gpurun_out/r6_l_${lib}_${rep}.err || { echo "bench $lib failed"; tail -20 gpurun_out/r6_l_${lib}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_l_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('${lib} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
