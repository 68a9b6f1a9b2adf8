# GPU parity (all -m gpu tests) then the quick c2..c5 bench of the default kernel
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/chk3 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/chk3/pytest_gpu.log 2>&1 || exit $?
for w in ${WORKLOADS:-c2 c3 c4 c5}; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > gpurun_out/chk3/$w.log 2>&1 || exit $?
done
