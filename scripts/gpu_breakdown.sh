# per-kernel breakdown of the single-pass path on c2/c3: default, loads only, +classification,
# stage A / stage B split (rocprofv3 kernel stats of scripts/ablate_scan.py)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in c2 c3; do
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/brk_$w -o run -- python3 $R/scripts/ablate_scan.py $w 1048576 0,1,2,3 > $O/brk_$w.log 2>&1 || exit $?
done
