#!/bin/bash
# Kernel trace + PMC passes of the head-kernel microbenchmark.
#   gpurun --timeout 900 -- bash scripts/gpu_headprof.sh TAG
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-hp}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/${TAG}_kt -o run -- \
  python vae-2_amd/tools/head_bench.py --iters 5 > gpurun_out/${TAG}_kt.log 2>&1 || exit $?
python - "$TAG" <<'EOF'
import csv, glob, sys
tag = sys.argv[1]
f = glob.glob(f"gpurun_out/{tag}_kt/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>5s} avg={float(r['AverageNs'])/1e3:9.1f}us")
EOF
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "upsum|head_|up_adj" -f csv \
    -d gpurun_out/${TAG}_pmc_$name -o run -- python vae-2_amd/tools/head_bench.py --iters 2 \
    > gpurun_out/${TAG}_pmc_$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
pass a SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE
pass b SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM
python - "$TAG" <<'EOF'
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
for name in ("a", "b"):
    fs = glob.glob(f"gpurun_out/{tag}_pmc_{name}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("no counters for pass", name); continue
    acc = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    for k, d in acc.items():
        n = len(cnt[k])
        print(k, " ".join(f"{c}={v / n:.3g}" for c, v in sorted(d.items())))
EOF
