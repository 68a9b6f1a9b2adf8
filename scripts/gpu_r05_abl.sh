# round 5: lean-kernel per-phase breakdown: event times and SQ instruction counts of the
# stage-A ablations (modes 15..18) beside the full kernel (mode 0), c2 and c3
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r05abl} && mkdir -p $O && export TMPDIR=/tmp
for wl in ${WLS:-c2 c3}; do
  timeout -k 10 240 python -u scripts/prof_modes.py --workload $wl --modes 0,15,16,17,18,0 --reps 5 > $O/time_$wl.log 2>&1 || { echo "time $wl failed"; tail -20 $O/time_$wl.log; exit 1; }
  cat $O/time_$wl.log | grep '"mode"'
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc1_$wl -o run -- python3 $R/scripts/prof_modes.py --workload $wl --modes 0,15,16,17,18 --reps 2 > $R/$O/pmc1_$wl.log 2>&1) || { echo "pmc1 $wl failed"; tail $R/$O/pmc1_$wl.log; exit 1; }
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT --output-format csv -d $R/$O/pmc2_$wl -o run -- python3 $R/scripts/prof_modes.py --workload $wl --modes 0,15,16,17,18 --reps 2 > $R/$O/pmc2_$wl.log 2>&1) || { echo "pmc2 $wl failed"; tail $R/$O/pmc2_$wl.log; exit 1; }
done
python3 scripts/pmc_summary.py $O/pmc1_* $O/pmc2_* 2>&1 | grep -E "==|scan_lean" > $O/sq_summary.txt
cat $O/sq_summary.txt
echo done
