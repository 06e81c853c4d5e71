#!/bin/bash
# Round 6: the 18-channel streaming 3x3 bounded to 128 VGPRs (__launch_bounds__(256, 4): 4
# workgroups per CU for every feature variant, as the LDS allows) -- stream tests, conv_bench
# and step A/B against the previous build (libvae2_hip_base.so), 3 interleaved reps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_dconv_stream_gpu.py > gpurun_out/r6_w_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6_w_tests.log; exit 1; }
tail -1 gpurun_out/r6_w_tests.log
for lib in new base; do
  if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
  VAE2_LIB=$PWD/$L timeout -k 10 120 python -u vae-2_amd/tools/conv_bench.py --only 3 --iters 50 > gpurun_out/r6_w_cb_$lib.log 2>&1 || { tail -20 gpurun_out/r6_w_cb_$lib.log; exit 1; }
  echo "== conv_bench $lib"; tail -3 gpurun_out/r6_w_cb_$lib.log
done
for rep in 1 2 3; do
  for lib in new base; do
    if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
    VAE2_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      > gpurun_out/r6_w_${lib}_${rep}.json 2> gpurun_out/r6_w_${lib}_${rep}.err || { echo "bench $lib failed"; tail -20 gpurun_out/r6_w_${lib}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_w_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('${lib} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
