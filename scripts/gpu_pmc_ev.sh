# SQ instruction-mix counters of the default single-pass kernel on c2 (two passes)
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $O/ev_pmcq1 -o run -- python3 $R/scripts/ablate_scan.py c2 1048576 0,30 > $O/ev_pmcq1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA --output-format csv -d $O/ev_pmcq2 -o run -- python3 $R/scripts/ablate_scan.py c2 1048576 0,30 > $O/ev_pmcq2.log 2>&1 || exit $?
cd $R && python scripts/pmc_summary.py $O/ev_pmcq1 $O/ev_pmcq2 > $O/ev_pmc_summary.txt
