#!/bin/bash
# SQ counters (3 passes) and HBM traffic (FETCH_SIZE / WRITE_SIZE) of the head up-sum
# kernels (head_bench --only upsum: upsum2_kernel and upsum_kernel) and of the
# 64 -> 256 1x1 GEMM (conv_bench shape 2), reduced by tools/sq_summary.py.
#   gpurun --timeout 900 -- bash scripts/gpu_r4_hpmc.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-hp}
mkdir -p gpurun_out
export TMPDIR=/tmp
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES"
G2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR"
G3="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM_RD SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_CYCLES_VMEM_WR"
G4="FETCH_SIZE"
G5="WRITE_SIZE"
p=0
for grp in "$G1" "$G2" "$G3" "$G4" "$G5"; do
  p=$((p+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "upsum" \
    -f csv -d gpurun_out/${TAG}_shb_p$p -o run -- python vae-2_amd/tools/head_bench.py \
    --only upsum --iters 3 > gpurun_out/${TAG}_shb_p$p.log 2>&1
  rc=$?; echo "upsum pass $p rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_shb_p$p.log; exit $rc; }
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-include-regex "gemm1x1" \
    -f csv -d gpurun_out/${TAG}_s2_p$p -o run -- python vae-2_amd/tools/conv_bench.py \
    --only 2 --iters 3 > gpurun_out/${TAG}_s2_p$p.log 2>&1
  rc=$?; echo "gemm1x1 pass $p rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_s2_p$p.log; exit $rc; }
done
python vae-2_amd/tools/sq_summary.py gpurun_out ${TAG} > gpurun_out/${TAG}_summary.json || exit 1
python - gpurun_out/${TAG}_summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    c, dv = v["counters"], v.get("derived", {})
    print(k[:70], {x: dv[x] for x in dv if "WAVE_CYCLES" in x or "/MFMA" in x},
          "fetch_MB", round(c.get("FETCH_SIZE", 0) / 1024, 1), "write_MB", round(c.get("WRITE_SIZE", 0) / 1024, 1),
          "waves", c.get("SQ_WAVES"), "vmem_wr", c.get("SQ_INSTS_VMEM_WR"))
PY
