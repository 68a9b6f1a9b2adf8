# multi-run tenant staging: GPU suite, bench c4, kernel stats
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/tenant && export TMPDIR=/tmp
O=gpurun_out/tenant
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c4 --no-cpu --no-pcie > $O/bench_c4.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o c4 -- python3 bench.py --workload c4 --no-cpu --no-pcie --steps 10 > $O/stats.log 2>&1 || exit $?
