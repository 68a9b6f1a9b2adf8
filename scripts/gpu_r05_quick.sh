# round 5: quick check of a kernel change: the GPU parity file, then event times and the
# SQ instruction mix of the lean kernel (modes 0, 15..18) on c2 / c3
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r05q} && mkdir -p $O && export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -10
[ $rc -eq 0 ] || exit 1
fi
for wl in ${WLS:-c2 c3}; do
  timeout -k 10 240 python -u scripts/prof_modes.py --workload $wl --modes ${MODES:-0,15,16,17,18,0} --reps 5 > $O/time_$wl.log 2>&1 || { echo "time $wl failed"; tail -20 $O/time_$wl.log; exit 1; }
  grep '"mode"' $O/time_$wl.log
  if [ -n "$PMC" ]; then
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc1_$wl -o run -- python3 $R/scripts/prof_modes.py --workload $wl --modes ${MODES:-0,15,16,17,18,0} --reps 2 > $R/$O/pmc1_$wl.log 2>&1) || { echo "pmc1 $wl failed"; tail $R/$O/pmc1_$wl.log; exit 1; }
  fi
  if [ -n "$TRAFFIC" ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/$O/pmc_${c}_$wl -o run -- python3 $R/scripts/prof_modes.py --workload $wl --modes 0 --reps 2 > $R/$O/pmc_${c}_$wl.log 2>&1) || { echo "pmc $c $wl failed"; tail $R/$O/pmc_${c}_$wl.log; exit 1; }
  done
  python3 scripts/pmc_summary.py $O/pmc_FETCH_SIZE_$wl $O/pmc_WRITE_SIZE_$wl 2>&1 | grep scan_lean
  fi
done
[ -n "$PMC" ] && python3 scripts/pmc_summary.py $O/pmc1_* 2>&1 | grep -E "==|scan_lean" | grep -E "==|VALU|SALU|LDS|VMEM|WAIT" > $O/sq_summary.txt && cat $O/sq_summary.txt
echo done
