# round 6: quick check of a kernel change: the GPU parity file (in-tree library), then for
# each variant library (VARS: scripts/var/libauthjx_<v>.so, built with -DAJX_LEAN_ABLATIONS)
# the event times of the lean kernel's modes (0, 15..18) and, with PMC=1, its SQ counts
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r06q} && mkdir -p $O && export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -4 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -10
[ $rc -eq 0 ] || exit 1
fi
for wl in ${WLS:-c2 c3}; do
  for v in ${VARS:-abl}; do
  timeout -k 10 240 python -u scripts/prof_modes.py --workload $wl --modes ${MODES:-0,15,16,17,18,0} --reps 5 --lib scripts/var/libauthjx_$v.so > $O/time_${wl}_$v.log 2>&1 || { echo "time $wl $v failed"; tail -20 $O/time_${wl}_$v.log; exit 1; }
  echo "$v $wl: $(grep -h '"mode"' $O/time_${wl}_$v.log | tr '\n' ' ')"
  if [ -n "$PMC" ]; then
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc1_${wl}_$v -o run -- python3 $R/scripts/prof_modes.py --workload $wl --modes ${MODES:-0,15,16,17,18} --reps 2 --lib $R/scripts/var/libauthjx_$v.so > $R/$O/pmc1_${wl}_$v.log 2>&1) || { echo "pmc1 $wl $v failed"; tail $R/$O/pmc1_${wl}_$v.log; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc1_${wl}_$v 2>&1 | grep -E "scan_lean" | grep -E "VALU|SALU|LDS|WAIT" > $O/sq_${wl}_$v.txt; cat $O/sq_${wl}_$v.txt
  fi
  done
done

for wl in $BENCH_WLS; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --cpu-seconds 3 --no-pcie --no-serve > $O/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail -20 $O/bench_$wl.log; exit 1; }
  tail -1 $O/bench_$wl.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$wl', d['ms_per_step'], d['value'], d.get('roofline',{}).get('frac'), d.get('parity'))"
done
echo bench-done
