#!/bin/bash
# Round 6: the 64-channel direct 3x3 (TM = TN = 4, 4 waves) bounded to 3 workgroups per CU
# (188 / 224 -> 128-158 VGPRs, no scratch; its 50 KB of LDS allows 3) vs the previous build
# (libvae2_hip_base.so) -- conv tests, conv_bench, step A/B (3 reps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py tests/test_bench_instances_gpu.py tests/test_lazy_bn_gpu.py \
  > gpurun_out/r6_dd_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r6_dd_tests.log | head -20; tail -5 gpurun_out/r6_dd_tests.log; exit 1; }
tail -1 gpurun_out/r6_dd_tests.log
for lib in new base; do
  if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
  VAE2_LIB=$PWD/$L timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 0 --iters 30 > gpurun_out/r6_dd_cb_$lib.log 2>&1 || { tail -20 gpurun_out/r6_dd_cb_$lib.log; exit 1; }
  echo "== conv_bench $lib"; tail -3 gpurun_out/r6_dd_cb_$lib.log
done
for rep in 1 2 3; do
  for lib in new base; do
    if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
    VAE2_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      > gpurun_out/r6_dd_${lib}_${rep}.json 2> gpurun_out/r6_dd_${lib}_${rep}.err || { echo "bench $lib failed"; tail -20 gpurun_out/r6_dd_${lib}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_dd_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('${lib} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
