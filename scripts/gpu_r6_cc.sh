#!/bin/bash
# Round 6: the quad fuse sum bounded to 3 waves per SIMD (139 VGPRs, no scratch) vs 198 VGPRs
# (libvae2_hip_base.so) -- fuse tests, step A/B (3 reps)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_kernels_gpu.py -k "fuse" > gpurun_out/r6_cc_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/r6_cc_tests.log; exit 1; }
tail -1 gpurun_out/r6_cc_tests.log
for rep in 1 2 3; do
  for lib in new base; do
    if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_base.so; fi
    VAE2_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      > gpurun_out/r6_cc_${lib}_${rep}.json 2> gpurun_out/r6_cc_${lib}_${rep}.err || { echo "bench $lib failed"; tail -20 gpurun_out/r6_cc_${lib}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_cc_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('${lib} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
