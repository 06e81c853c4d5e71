#!/bin/bash
# Streaming direct 3x3: tune sweep (LDS vs global weights, workgroups per CU) on the 18 / 36
# channel conv_bench shapes, then the stream tests.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 9=0 9=2 9=2,11=0 9=2,11=0,10=2 9=2,11=0,10=4 9=2,10=2 9=2,10=4 9=2,10=1 9=2,11=0,10=1; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 --iters 20 --tune $t \
    > gpurun_out/r5m_conv_$t.log 2>&1 || { tail -5 gpurun_out/r5m_conv_$t.log; exit 1; }
  echo "== conv tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5m_conv_$t.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_dconv_stream_gpu.py \
  > gpurun_out/r5m_stream.log 2>&1
rc=$?; echo "stream tests rc=$rc"; tail -2 gpurun_out/r5m_stream.log
