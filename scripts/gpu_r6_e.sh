#!/bin/bash
# Round 6: BN reduce blocks sized by whole passes -- microbench + step A/B against the
# round-5 BN kernels (libvae2_hip_r5bn.so), BN parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_lazy_bn_gpu.py tests/test_kernels_gpu.py tests/test_model_gpu.py -k "bn or BN or elbo_step or w18 or lazy or resbn" \
  > gpurun_out/r6_e_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r6_e_tests.log; exit 1; }
tail -2 gpurun_out/r6_e_tests.log
for lib in new r5bn; do
  if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_r5bn.so; fi
  VAE2_LIB=$PWD/$L timeout -k 10 120 python -u vae-2_amd/tools/bn_bench.py --iters 50 > gpurun_out/r6_e_bnbench_$lib.txt 2>&1 || { echo "bn_bench $lib failed"; tail gpurun_out/r6_e_bnbench_$lib.txt; exit 1; }
  echo "== bn_bench $lib"; cat gpurun_out/r6_e_bnbench_$lib.txt | tail -12
done
for rep in 1 2; do
  for lib in new r5bn; do
    if [ $lib = new ]; then L=vae-2_amd/vae2/libvae2_hip.so; else L=vae-2_amd/vae2/libvae2_hip_r5bn.so; fi
    VAE2_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-roofline \
      > gpurun_out/r6_e_${lib}_${rep}.json 2> gpurun_out/r6_e_${lib}_${rep}.err || { echo "bench $lib failed"; tail -20 gpurun_out/r6_e_${lib}_${rep}.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/r6_e_${lib}_${rep}.json').read().strip().splitlines()[-1]); print('${lib} rep ${rep}:', d['value'], 'frames/s', d['ms_per_step'], 'ms/step')"
  done
done
