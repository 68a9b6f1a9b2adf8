# Round evidence on one MI355X: GPU parity tests, smoke, PMC passes for HBM bytes of the
# headline kernel (FETCH_SIZE / WRITE_SIZE, separate runs), then the bench lines (c2 headline
# with that traffic, c3, c4, c5) and rocprofv3 kernel-trace stats of the c2 / c3 benches.
# Every GPU step has its own time limit; the first failure ends the script.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu > $O/pmc_write.log 2>&1 || exit $?
cd $R
python scripts/pmc_traffic.py $O/pmc_fetch $O/pmc_write c2 1048576 profiles/pmc_traffic.json > $O/pmc_traffic.log 2>&1 || exit $?
cp profiles/pmc_traffic.json $O/pmc_traffic.json
timeout -k 10 600 python bench.py > $O/bench_c2.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c3 > $O/bench_c3.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c4 --steps 10 > $O/bench_c4.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c5 --steps 10 > $O/bench_c5.log 2>&1 || exit $?
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o run -- python3 $R/bench.py --no-cpu > $O/prof_c2.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o run -- python3 $R/bench.py --workload c3 --no-cpu > $O/prof_c3.log 2>&1 || exit $?
echo done > $O/round_ok
