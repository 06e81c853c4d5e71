#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/r16_counters.txt 2>&1
echo "list rc=$?"
pass() { local name=$1; shift; echo "== pass $name: $*"; timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "igemm|wgrad" -f csv -d gpurun_out/r16_pmc_$name -o run -- python vae-2_amd/tools/conv_bench.py --only 3 0 --iters 3 > gpurun_out/r16_pmc_$name.log 2>&1; local rc=$?; echo "rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY
pass b SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS
pass c SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES
pass d TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
pass e GRBM_GUI_ACTIVE SQ_WAIT_ANY SQ_INST_CYCLES_VMEM TA_BUSY_avr
ls gpurun_out | grep r16
