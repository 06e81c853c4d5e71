#!/bin/bash
# Round 5: narrow direct-3x3 phase ablations (no stores + no MFMA loop; + no staging loads)
# and dconv3 vs the gather kernel per narrow shape; the IPC SyncBN test with graph latency.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in libvae2_hip.so libvae2_hip_abl6.so libvae2_hip_abl7.so; do
  VAE2_LIB=$PWD/vae-2_amd/vae2/$lib timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 6 \
    --iters 20 > gpurun_out/r5f_conv_$lib.log 2>&1 || { tail -20 gpurun_out/r5f_conv_$lib.log; exit 1; }
  echo "== $lib"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5f_conv_$lib.log
done
timeout -k 10 200 python vae-2_amd/tools/conv_bench.py --only 3 4 5 6 --iters 20 --algo 0 1 2 \
  > gpurun_out/r5f_conv_algo.log 2>&1 || { tail -20 gpurun_out/r5f_conv_algo.log; exit 1; }
grep -E "^==|^[0-9]+x[0-9]+" gpurun_out/r5f_conv_algo.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_syncbn_ipc_gpu.py -s \
  > gpurun_out/r5f_ipc.log 2>&1
rc=$?; echo "ipc rc=$rc"; grep -E "rank|passed|failed" gpurun_out/r5f_ipc.log
