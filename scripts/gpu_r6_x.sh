#!/bin/bash
# Round 6: why the narrow multi-layer BatchNorm backward apply (18@128x256
# + 36@64x128 + 72@32x64) runs below the wide one (64@128x256) -- bn_bench timings and SQ PMC
# of bn_bwd_apply_multi_kernel for both sets (one rocprofv3 --pmc pass per counter group)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for set in narrow wide; do
  timeout -k 10 120 python -u vae-2_amd/tools/bn_bench.py --set $set --res 0 > gpurun_out/r6_x_bench_$set.txt 2>&1 || { tail gpurun_out/r6_x_bench_$set.txt; exit 1; }
  echo "== $set"; cat gpurun_out/r6_x_bench_$set.txt
done
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r6_x_counters.txt 2>&1
grep -o "[A-Z][A-Z_0-9]*" gpurun_out/r6_x_counters.txt | sort -u > gpurun_out/r6_x_names.txt
i=0
for grp0 in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_VALU" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_BRANCH" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  grp=""
  for c in $grp0; do grep -qx "$c" gpurun_out/r6_x_names.txt && grp="$grp $c"; done
  echo "pass $i:$grp"
  for set in narrow wide; do
    timeout -s KILL 90 rocprofv3 --pmc $grp --kernel-include-regex bn_bwd_apply_multi -f csv \
      -d gpurun_out/r6_x_${set}_p$i -o run -- python vae-2_amd/tools/bn_bench.py --set $set --res 0 \
      --only bwd_apply --iters 5 > gpurun_out/r6_x_${set}_p$i.log 2>&1
    rc=$?; echo "pass $i $set rc=$rc"
    [ $rc -ne 0 ] && { tail -5 gpurun_out/r6_x_${set}_p$i.log; exit $rc; }
  done
done
exit 0
