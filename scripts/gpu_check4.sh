# GPU parity tests (incl. `#` count selectors) and smoke on the current tree
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/chk4 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/chk4/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/chk4/smoke.log 2>&1 || exit $?
