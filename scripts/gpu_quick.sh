# one iteration: GPU parity tests, then the default kernel on c2 / c3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python scripts/ablate_scan.py c2 1048576 0 > gpurun_out/variants.log 2>&1 || exit $?
timeout -k 10 200 python scripts/ablate_scan.py c3 1048576 0 >> gpurun_out/variants.log 2>&1 || exit $?
