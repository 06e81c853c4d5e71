#!/bin/bash
# Round-5 first call: sanity bench at HEAD, narrow-conv phase ablations (VAE2_ABLATE
# builds), then the world-1 RCCL graph-capture probe (bounded, stack dumps on a hang).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 10 > gpurun_out/r5a_bench.log 2>&1 \
  || { tail -20 gpurun_out/r5a_bench.log; exit 1; }
grep '^{' gpurun_out/r5a_bench.log | cut -c1-200
for lib in libvae2_hip.so libvae2_hip_abl1.so libvae2_hip_abl4.so; do
  VAE2_LIB=$PWD/vae-2_amd/vae2/$lib timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 6 7 \
    --iters 20 > gpurun_out/r5a_conv_$lib.log 2>&1 || { tail -20 gpurun_out/r5a_conv_$lib.log; exit 1; }
  echo "== $lib"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5a_conv_$lib.log
done
timeout -k 10 240 python -u vae-2_amd/tools/dist_step_probe.py --graph --steps 3 --dump-after 50 \
  > gpurun_out/r5a_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -40 gpurun_out/r5a_probe.log
