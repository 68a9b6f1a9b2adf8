# lane kernel iteration: GPU parity, then c2 timing of the default build, occupancy
# variants and ablations
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lane2 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lane2/pytest_gpu.log 2>&1 || exit $?
for m in 0 24 23 22; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --steps 10 --kernel-mode $m > gpurun_out/lane2/c2_m$m.log 2>&1 || exit $?
done
for v in w2 w3; do
  AUTHJX_LIB=$PWD/scripts/bin/libauthjx_$v.so timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --steps 10 > gpurun_out/lane2/c2_$v.log 2>&1 || exit $?
done
timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --steps 10 --workload c3 > gpurun_out/lane2/c3_m0.log 2>&1 || exit $?
