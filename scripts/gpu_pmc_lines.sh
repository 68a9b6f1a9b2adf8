# SQ counters of the line engine on c2 (two passes)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/pmcl1 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $O/pmcl1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_IFETCH SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES --output-format csv -d $O/pmcl2 -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu > $O/pmcl2.log 2>&1 || exit $?
