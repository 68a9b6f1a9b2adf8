# quick check of the current tree: GPU suite, then bench lines for c2..c5 (no CPU legs)
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-quick} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for w in c2 c3 c4 c5; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu --no-pcie > $O/bench_$w.log 2>&1 || exit $?
done
