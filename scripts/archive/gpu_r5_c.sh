#!/bin/bash
# Round 5: narrow weight-gradient kernel tests + per-shape A/B (tune key 7), the RCCL graph
# capture (probe + restored test), the step A/B, then SQ counters of the BN backward apply.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_wgrad_narrow_gpu.py \
  > gpurun_out/r5c_wn_tests.log 2>&1
rc=$?; echo "narrow wgrad tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/r5c_wn_tests.log | head -30
[ $rc -ne 0 ] && exit $rc
for t in 7=0 7=1 7=2; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only 3 4 5 --iters 20 --tune $t \
    > gpurun_out/r5c_conv_$t.log 2>&1 || { tail -5 gpurun_out/r5c_conv_$t.log; exit 1; }
  echo "== tune $t"; grep -E "^[0-9]+x[0-9]+" gpurun_out/r5c_conv_$t.log
done
for t in 7=0 7=1 7=0 7=1; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --steps 20 --conv-tune $t \
    > gpurun_out/r5c_bench_$t.log 2>&1 || { tail -20 gpurun_out/r5c_bench_$t.log; exit 1; }
  echo "[bench tune $t] $(grep '^{' gpurun_out/r5c_bench_$t.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 240 python -u vae-2_amd/tools/dist_step_probe.py --graph --steps 3 --dump-after 50 \
  > gpurun_out/r5c_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -E "eager|step|graph ==|probe ok|Error|error" gpurun_out/r5c_probe.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_rccl_gpu.py \
  > gpurun_out/r5c_rccl_tests.log 2>&1
rc=$?; echo "rccl tests rc=$rc"; tail -5 gpurun_out/r5c_rccl_tests.log
[ $rc -ne 0 ] && exit $rc
rocprofv3 -L > gpurun_out/r5c_counters.txt 2>&1
echo "counter list: $(wc -l < gpurun_out/r5c_counters.txt) lines"
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU"
timeout -s KILL 150 rocprofv3 --pmc $G1 --kernel-include-regex "bn_bwd_apply_multi" -f csv \
  -d gpurun_out/r5c_bnsq1 -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline \
  --no-roofline --graph off > gpurun_out/r5c_bnsq1.log 2>&1
echo "bn sq pass rc=$?"
