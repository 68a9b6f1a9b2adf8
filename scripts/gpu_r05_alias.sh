# round 5: the lean kernel with its documents cache-resident (request i reads document i % K)
# beside the normal batch: how much of each phase is HBM access shape, how much issue
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r05alias} && mkdir -p $O && export TMPDIR=/tmp
for wl in ${WLS:-c2 c3}; do
  for k in ${ALIASES:-0 2048}; do
    timeout -k 10 240 python -u scripts/prof_modes.py --workload $wl --alias $k --modes ${MODES:-0,15,16,17,18,0} --reps 5 > $O/time_${wl}_$k.log 2>&1 || { echo "time $wl $k failed"; tail -20 $O/time_${wl}_$k.log; exit 1; }
    grep '"mode"' $O/time_${wl}_$k.log
  done
done
echo done
