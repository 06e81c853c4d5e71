#!/bin/bash
# Round 5: the RCCL graph capture in thread-local mode (probe + restored test), then SQ
# counters of the BatchNorm backward apply launches in the eager step, and the counter list.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -u vae-2_amd/tools/dist_step_probe.py --graph --steps 3 --dump-after 50 \
  > gpurun_out/r5b_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -E "eager|step|graph ==|probe ok|Error|error" gpurun_out/r5b_probe.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dist_rccl_gpu.py \
  > gpurun_out/r5b_rccl_tests.log 2>&1
rc=$?; echo "rccl tests rc=$rc"; tail -5 gpurun_out/r5b_rccl_tests.log
[ $rc -ne 0 ] && exit $rc
rocprofv3 -L > gpurun_out/r5b_counters.txt 2>&1 || rocprofv3 --list-avail > gpurun_out/r5b_counters.txt 2>&1
echo "counter list: $(wc -l < gpurun_out/r5b_counters.txt) lines"
G1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU"
timeout -s KILL 150 rocprofv3 --pmc $G1 --kernel-include-regex "bn_bwd_apply_multi|bn_apply_multi" -f csv \
  -d gpurun_out/r5b_bnsq1 -o run -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline \
  --no-roofline --graph off > gpurun_out/r5b_bnsq1.log 2>&1
echo "bn sq pass rc=$?"
