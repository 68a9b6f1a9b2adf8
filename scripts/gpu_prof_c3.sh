# per-kernel times and counters for the c3 workload (split path)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c3 -o run -- python3 $R/bench.py --workload c3 --steps 5 --warmup 1 --no-cpu > $R/gpurun_out/prof_c3.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/pmc_c3 -o run -- python3 $R/bench.py --workload c3 --steps 2 --warmup 1 --no-cpu > $R/gpurun_out/pmc_c3.log 2>&1
