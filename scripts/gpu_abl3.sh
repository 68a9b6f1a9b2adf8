# stage-B share of the fused kernel (NOB variant) and the FETCH calibration of the
# per-lane 16-B load pattern (loads-only ablation, mode 1) on c2
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/abl3 && export TMPDIR=/tmp
O=gpurun_out/abl3
timeout -k 10 200 python scripts/ablate_scan.py c2 1048576 0,1 > $O/base.log 2>&1 || exit $?
AUTHJX_LIB=$PWD/scripts/var/libauthjx_nob.so timeout -k 10 200 python scripts/ablate_scan.py c2 1048576 0 > $O/nob.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch1 -o f -- python3 bench.py --workload c2 --no-cpu --no-pcie --steps 2 --warmup 1 --kernel-mode 1 > $O/fetch1.log 2>&1 || exit $?
AUTHJX_LIB=$PWD/scripts/var/libauthjx_nob.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetchnob -o f -- python3 bench.py --workload c2 --no-cpu --no-pcie --steps 2 --warmup 1 > $O/fetchnob.log 2>&1 || exit $?
