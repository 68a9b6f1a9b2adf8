# wave-interleaved capture rows: GPU suite, bench c2/c5, FETCH/WRITE passes on c2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/rows && export TMPDIR=/tmp
O=gpurun_out/rows
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c2 --no-cpu --no-pcie > $O/bench_c2.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload c5 --no-cpu > $O/bench_c5.log 2>&1 || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/stats -o run -- python3 bench.py --workload c2 --no-cpu --no-pcie --steps 10 > $O/stats.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o f -- python3 bench.py --workload c2 --no-cpu --no-pcie --steps 2 --warmup 1 > $O/fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $O/write -o w -- python3 bench.py --workload c2 --no-cpu --no-pcie --steps 2 --warmup 1 > $O/write.log 2>&1 || exit $?
