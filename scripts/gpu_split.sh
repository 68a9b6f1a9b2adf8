# per-kernel split of the fast path (mode 3: stage A and stage B as two launches) on c2
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_split -o run -- python3 $R/scripts/ablate_scan.py c2 > $O/prof_split.log 2>&1 || exit $?
