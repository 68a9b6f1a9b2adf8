# GPU parity tests, then sorted (0) vs unsorted (100) timing on c5 / c2 / c3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
cd $R && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python3 $R/scripts/ablate_scan.py c5 1048576 0,100 > $O/brk_c5.log 2>&1 || exit $?
timeout -k 10 200 python3 $R/scripts/ablate_scan.py c2 1048576 0,100 >> $O/brk_c5.log 2>&1 || exit $?
timeout -k 10 200 python3 $R/scripts/ablate_scan.py c3 1048576 0,100 >> $O/brk_c5.log 2>&1 || exit $?
