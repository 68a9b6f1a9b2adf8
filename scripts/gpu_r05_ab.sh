# round 5: A/B of kernel variants in one box: the in-tree library and scripts/var builds
# (VARS), c2 / c3 event times, alternating runs
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r05ab} && mkdir -p $O && export TMPDIR=/tmp
for wl in ${WLS:-c2 c3}; do
  for rep in 1 2; do
    timeout -k 10 240 python -u scripts/prof_modes.py --workload $wl --modes ${MODES:-0} --reps 10 > $O/t_${wl}_main_$rep.log 2>&1 || { echo "main $wl failed"; tail -5 $O/t_${wl}_main_$rep.log; exit 1; }
    echo "main $wl $(grep -h '"mode"' $O/t_${wl}_main_$rep.log | tr '\n' ' ')"
    for v in $VARS; do
      timeout -k 10 240 python -u scripts/prof_modes.py --workload $wl --modes ${MODES:-0} --reps 10 --lib scripts/var/libauthjx_$v.so > $O/t_${wl}_${v}_$rep.log 2>&1 || { echo "$v $wl failed"; tail -5 $O/t_${wl}_${v}_$rep.log; exit 1; }
      echo "$v $wl $(grep -h '"mode"' $O/t_${wl}_${v}_$rep.log | tr '\n' ' ')"
    done
  done
done
echo done
