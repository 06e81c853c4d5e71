#!/bin/bash
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
pass() { local name=$1; shift; echo "== pass $name: $*"; timeout -k 10 300 rocprofv3 --pmc "$@" --kernel-include-regex "dconv3|wgrad3" -f csv -d gpurun_out/r22_pmc_$name -o run -- python vae-2_amd/tools/conv_bench.py --only 3 0 --iters 3 > gpurun_out/r22_pmc_$name.log 2>&1; local rc=$?; echo "rc=$rc"; case $rc in 124|134|137|139) exit $rc;; esac; }
pass a SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
pass b SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
pass c SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY
pass d SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY
pass e TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
