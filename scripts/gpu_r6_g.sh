#!/bin/bash
# Round 6: the default bench line with the live rocprofv3 passes (PMC traffic + trace
# average of the dominant kernel measured inside bench.py), timed end to end
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
t0=$(date +%s)
timeout -k 10 900 python -u bench.py > gpurun_out/r6_g_bench.json 2> gpurun_out/r6_g_bench.err || { echo "bench failed"; tail -30 gpurun_out/r6_g_bench.err; exit 1; }
t1=$(date +%s)
echo "bench wall $((t1 - t0)) s"
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6_g_bench.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"])
r = d["roofline"]
print({k: r[k] for k in ("kernel", "avg_launch_us", "achieved", "frac", "traffic", "traffic_unit") if k in r})
print(r.get("trace"), r.get("traffic_over_algorithmic"), r.get("conv_stack", {}).get("frac"))
print(d.get("cpu_baseline"))
PY
