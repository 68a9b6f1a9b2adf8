# round-2 check: GPU parity (default single-pass kernel + lane kernel test), c2/c3 bench
# of both kernels
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/chk2 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/chk2/pytest_gpu.log 2>&1 || exit $?
for w in c2 c3; do for m in 0 20; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $w --kernel-mode $m > gpurun_out/chk2/${w}_m$m.log 2>&1 || exit $?
done; done
