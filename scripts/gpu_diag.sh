# stage-A ablations (loads only / loads+classify / full / split) and one SQ counter pass on c2
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd $R
timeout -k 10 300 python scripts/ablate_scan.py c2 > $O/ablate.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/pmc_sq1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $O/pmc_sq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/pmc_sq2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $O/pmc_sq2.log 2>&1 || exit $?
