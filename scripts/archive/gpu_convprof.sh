#!/bin/bash
# Kernel trace + PMC passes of the conv microbenchmark for selected shapes.
#   gpurun --timeout 900 -- bash scripts/gpu_convprof.sh TAG "3 4" "dconv3|igemm|wgrad"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-cp}
ONLY=${2:-3}
RX=${3:-"dconv3|igemm|wgrad"}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python vae-2_amd/tools/conv_bench.py --only $ONLY --iters 10 $EXTRA \
  > gpurun_out/${TAG}_bench.log 2>&1 || { tail gpurun_out/${TAG}_bench.log; exit 1; }
cat gpurun_out/${TAG}_bench.log
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex "$RX" -f csv \
    -d gpurun_out/${TAG}_pmc_$name -o run -- python vae-2_amd/tools/conv_bench.py --only $ONLY --iters 2 $EXTRA \
    > gpurun_out/${TAG}_pmc_$name.log 2>&1
  local rc=$?; echo "pass $name rc=$rc"
  case $rc in 124|134|137|139) exit $rc;; esac
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass b SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE
python - "$TAG" <<'PY'
import csv, glob, sys
from collections import defaultdict
tag = sys.argv[1]
for name in ("a", "b"):
    fs = glob.glob(f"gpurun_out/{tag}_pmc_{name}/**/*counter_collection.csv", recursive=True)
    if not fs:
        print("no counters for pass", name); continue
    acc = defaultdict(lambda: defaultdict(float)); cnt = defaultdict(set)
    for r in csv.DictReader(open(fs[0])):
        k = r["Kernel_Name"].split("(")[0][-45:]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    for k, d in acc.items():
        n = len(cnt[k])
        print(k, " ".join(f"{c}={v / n:.3g}" for c, v in sorted(d.items())))
PY
