#!/bin/bash
# Diagnose the bf16 trajectory test under the 18-channel gather remainder (key 6 = 2):
# fp32 losses of the 6-step Adam run with key 6 = 0 / 2, then the fp32 parity suites.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
cd tests
timeout -k 10 300 python - > ../gpurun_out/r5hh_traj.log 2>&1 <<'PY'
import sys
sys.path.insert(0, ".")
import conftest  # noqa: F401  (paths)
from test_bf16_gpu import _inputs, _run
from vae2 import _lib
lib = _lib.load()
xs, eps, code = _inputs()
xs = [0.1 * x for x in xs]
for k6 in (0, 2, 0, 2):
    lib.vae2_conv2d_set_tune(6, k6)
    h32, _ = _run(False, xs, eps, code, steps=6, lr=3e-3)
    print("key6", k6, "fp32", [round(h[0], 2) for h in h32], flush=True)
lib.vae2_conv2d_set_tune(6, 2)
h16, _ = _run(True, xs, eps, code, steps=6, lr=3e-3)
print("bf16", [round(h[0], 2) for h in h16], flush=True)
PY
rc=$?; cd ..; echo "traj rc=$rc"; cat gpurun_out/r5hh_traj.log | grep -E "key6|bf16|Error" | head
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py \
  tests/test_bench_instances_gpu.py tests/test_kernels_gpu.py > gpurun_out/r5hh_tests.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/r5hh_tests.log
