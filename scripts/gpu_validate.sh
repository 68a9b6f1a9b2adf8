# validate the committed tree: GPU parity tests, smoke, quick c2..c5 bench lines
set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/val && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/val/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/val/smoke.log 2>&1 || exit $?
for w in c2 c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > gpurun_out/val/$w.log 2>&1 || exit $?
done
