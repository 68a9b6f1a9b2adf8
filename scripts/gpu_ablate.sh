# fast-path ablations on c2 and c3 (see scripts/ablate_scan.py)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python scripts/ablate_scan.py c2 > gpurun_out/ablate.log 2>&1 || exit $?
timeout -k 10 300 python scripts/ablate_scan.py c3 >> gpurun_out/ablate.log 2>&1 || exit $?
