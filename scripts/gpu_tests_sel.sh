cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_train_cli_gpu.py -k "modes or gan or w18_backward or bench_geometry or deferred or train_cli" > gpurun_out/gt1.log 2>&1
rc=$?; tail -30 gpurun_out/gt1.log; exit $rc
