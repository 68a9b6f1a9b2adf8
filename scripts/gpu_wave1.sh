# first GPU run of the wave kernel: parity tests, then c2/c3 bench (wave vs round-1 kernel)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/wave1 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/wave1/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie > gpurun_out/wave1/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --kernel-mode 6 > gpurun_out/wave1/bench_c2_old.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --workload c3 > gpurun_out/wave1/bench_c3.log 2>&1 || exit $?
