#!/bin/bash
# Selected GPU tests (no -x) + direct-3x3 ablation timings (diagnostic builds in abl/).
#   gpurun -- bash scripts/gpu_abl.sh "<pytest -k expression>" "<conv_bench --only indices>"
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
if [ -n "$1" ]; then
  timeout -k 10 900 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests -m gpu \
    -k "$1" > gpurun_out/gt2.log 2>&1
  grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/gt2.log | tail -30
fi
for lib in vae-2_amd/vae2/libvae2_hip.so abl/libvae2_hip_a1.so abl/libvae2_hip_a2.so abl/libvae2_hip_a3.so; do
  echo "== $lib"
  VAE2_LIB=$PWD/$lib timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only $2 --iters 30 \
    --algo 0 2>&1 | grep -v "^per-step\|^  \|weighted\|== algo" || exit 1
done
