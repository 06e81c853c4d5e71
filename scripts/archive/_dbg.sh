cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export VAE2_UPSUM_DEBUG=7
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "upsum|head_out_bwd_apply" -f csv \
    -d gpurun_out/dbg_pmc_$name -o run -- python vae-2_amd/tools/head_bench.py --iters 2 \
    > gpurun_out/dbg_pmc_$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT
pass b SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM
pass c TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
pass d SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_BRANCH
python - <<'PY'
import csv, glob
from collections import defaultdict
for name in "abcd":
    fs = glob.glob(f"gpurun_out/dbg_pmc_{name}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("no counters for pass", name); continue
    acc = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"][:30]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    for k, d in acc.items():
        n = len(cnt[k])
        print(k, " ".join(f"{c}={v / n:.3g}" for c, v in sorted(d.items())))
PY
