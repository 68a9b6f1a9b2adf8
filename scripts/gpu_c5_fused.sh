# c5 with the response selectors captured by the forest's own scan: GPU parity tests,
# the c5 bench line and its rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c5 --steps 10 > gpurun_out/bench_c5.log 2>&1 || exit $?
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5 -o run -- python3 $R/bench.py --workload c5 --steps 10 --no-cpu > $O/prof_c5.log 2>&1 || exit $?
