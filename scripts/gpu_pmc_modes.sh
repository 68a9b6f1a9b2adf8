# HBM bytes (FETCH_SIZE / WRITE_SIZE passes) per kernel variant on c2: modes 0, 5, 3
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for C in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv -d $O/pmcm_$C -o run -- python3 $R/scripts/ablate_scan.py c2 1048576 0,5,3 > $O/pmcm_$C.log 2>&1 || exit $?
done
