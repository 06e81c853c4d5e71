#!/bin/bash
# SQ issue / stall counters of the dconv3 kernels on one conv_bench shape, one rocprofv3
# --pmc pass per counter group (<= 8 SQ counters each).
#   gpurun -- bash scripts/gpu_sqpmc.sh TAG "<conv_bench --only idx>" "<kernel regex>"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-sq}
ONLY=${2:-3}
REGEX=${3:-dconv3_kernel}
EXTRA=${4:-}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${TAG}_counters.txt 2>&1
grep -o "SQ_[A-Z_0-9]*" gpurun_out/${TAG}_counters.txt | sort -u > gpurun_out/${TAG}_sq_names.txt
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_LDS_UNALIGNED_STALL"; do
  i=$((i+1))
  ok=""
  for c in $grp; do grep -qx "$c" gpurun_out/${TAG}_sq_names.txt && ok="$ok $c"; done
  echo "pass $i:$ok"
  timeout -s KILL 120 rocprofv3 --pmc $ok --kernel-include-regex "$REGEX" -f csv \
    -d gpurun_out/${TAG}_p$i -o run -- python vae-2_amd/tools/conv_bench.py --only $ONLY \
    --iters 5 $EXTRA > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; }
done
exit 0
