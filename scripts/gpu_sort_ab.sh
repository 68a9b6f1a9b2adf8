# parity with the length-bucketed order + A/B timing (0 = sorted, 100 = unsorted) on c2/c3
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python scripts/ablate_scan.py c2 1048576 0,100 > $O/ab.log 2>&1 || exit $?
timeout -k 10 200 python scripts/ablate_scan.py c3 1048576 0,100 >> $O/ab.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ablate_scan.py c4 2097152 0,100,200 >> $O/ab.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_sort -o run -- python3 $R/scripts/ablate_scan.py c2 1048576 0 > $O/prof_sort.log 2>&1 || exit $?
