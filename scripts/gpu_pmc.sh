#!/bin/bash
# HBM traffic of one kernel of the bench from two separate rocprofv3 --pmc passes
# (FETCH_SIZE, then WRITE_SIZE; MI355X_MICROARCH.md §HBM), reduced by tools/pmc_traffic.py.
#   gpurun --timeout 600 -- bash scripts/gpu_pmc.sh TAG "dconv3_kernel<4, 4, false>"
cd "$GRAFT_REPO_ROOT" || exit 1
TAG=${1:-pmc}
KERNEL=${2:-"dconv3_kernel<4, 4, false>"}
mkdir -p gpurun_out
export TMPDIR=/tmp
REGEX=$(printf '%s' "$KERNEL" | sed 's/[<>]/./g')
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-include-regex "$REGEX" -f csv \
    -d gpurun_out/${TAG}_$c -o run -- python bench.py --steps 1 --warmup 1 \
    --no-cpu-baseline --no-roofline --graph off > gpurun_out/${TAG}_$c.log 2>&1
  rc=$?; echo "pass $c rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/${TAG}_$c.log; exit $rc; }
done
python vae-2_amd/tools/pmc_traffic.py --fetch gpurun_out/${TAG}_FETCH_SIZE \
  --write gpurun_out/${TAG}_WRITE_SIZE --kernel "$KERNEL" --out gpurun_out/${TAG}_pmc_traffic.json
