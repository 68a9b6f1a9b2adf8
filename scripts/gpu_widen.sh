# GPU parity tests (incl. c4 multi-tenant, select spans, c5 full phase) + the c4 bench line
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --workload c4 --steps 10 > $O/bench_c4.log 2>&1 || exit $?
echo done > $O/widen_ok
