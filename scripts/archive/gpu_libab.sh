#!/bin/bash
# bench.py against alternative builds of the library (VAE2_LIB), same box, in turn.
#   gpurun -- bash scripts/gpu_libab.sh libvae2_hip.so libvae2_hip_nt1.so ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
i=0
for lib in "$@" "$@"; do
  i=$((i+1))
  VAE2_LIB=$PWD/vae-2_amd/vae2/$lib timeout -k 10 300 python bench.py --no-cpu-baseline \
    --no-roofline --steps 20 > gpurun_out/libab_$i.log 2>&1 || { tail -20 gpurun_out/libab_$i.log; exit 1; }
  echo "[$lib] $(grep '^{' gpurun_out/libab_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
