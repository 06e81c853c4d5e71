#!/bin/bash
# SQ issue / stall counters (3 rocprofv3 --pmc passes, <= 8 SQ counters each) of the conv
# kernels of the narrow conv_bench shapes, reduced to one JSON, plus a batch scan of the
# per-launch times (fixed cost per launch).
#   gpurun --timeout 900 -- bash scripts/gpu_narrow_pmc.sh TAG "3 4 5 9"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-npmc}
IDX=${2:-"3 4 5 9"}
mkdir -p gpurun_out
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR"
G3="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_WR"
for i in $IDX; do
  p=0
  for grp in "$G1" "$G2" "$G3"; do
    p=$((p+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "dconv3|wgrad3|igemm|wgrad_kernel|gemm1x1" \
      -f csv -d gpurun_out/${TAG}_s${i}_p$p -o run -- python vae-2_amd/tools/conv_bench.py \
      --only $i --iters 5 > gpurun_out/${TAG}_s${i}_p$p.log 2>&1
    rc=$?; echo "shape $i pass $p rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_s${i}_p$p.log; exit $rc; }
  done
done
python vae-2_amd/tools/sq_summary.py gpurun_out ${TAG} > gpurun_out/${TAG}_summary.json || exit 1
for b in 4 8 16; do
  timeout -k 10 120 python vae-2_amd/tools/conv_bench.py --only $IDX --batch $b --iters 20 \
    > gpurun_out/${TAG}_batch$b.log 2>&1 || { tail -5 gpurun_out/${TAG}_batch$b.log; exit 1; }
  echo "B=$b"; grep -E "^[0-9]+x[0-9]+" gpurun_out/${TAG}_batch$b.log
done
