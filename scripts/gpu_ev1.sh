# event scanner first GPU run: parity tests, then token (30) vs event (0) scanner timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ev1 && export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/ev1/pytest_gpu.log 2>&1 || exit $?
for w in c2 c3 c5; do
  timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0,30 > gpurun_out/ev1/ab_$w.log 2>&1 || exit $?
done
timeout -k 10 200 python scripts/ablate_scan.py c4 2097152 0,30 > gpurun_out/ev1/ab_c4.log 2>&1 || exit $?
