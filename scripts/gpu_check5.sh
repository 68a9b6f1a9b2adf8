cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/chk5 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -k "alternative or count" > gpurun_out/chk5/pytest_gpu.log 2>&1 || exit $?
