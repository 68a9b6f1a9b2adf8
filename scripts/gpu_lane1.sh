# first GPU run of the lane kernel: parity tests (default kernel = lane), then c2/c3
# bench A/B against the round-1 kernel (mode 6) and the staging-only ablation (mode 21)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/lane1 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/lane1/pytest_gpu.log 2>&1 || exit $?
for m in 0 6 21 10; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --kernel-mode $m > gpurun_out/lane1/bench_c2_m$m.log 2>&1 || exit $?
done
for m in 0 6; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --workload c3 --kernel-mode $m > gpurun_out/lane1/bench_c3_m$m.log 2>&1 || exit $?
done
