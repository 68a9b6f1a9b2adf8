# stage A / stage B split (mode 3: two launches) against the single-pass kernel
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/split && export TMPDIR=/tmp
for w in c2 c3; do
  timeout -k 10 200 python scripts/ablate_scan.py $w 1048576 0,3 > gpurun_out/split/ab_$w.log 2>&1 || exit $?
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/split/st_c3 -o c3 -- python3 $GRAFT_REPO_ROOT/scripts/ablate_scan.py c3 1048576 3 > $GRAFT_REPO_ROOT/gpurun_out/split/st_c3.log 2>&1 || exit $?
