# round 4: the streaming kernel (default) vs the lean kernel (--kernel-mode 41) and the
# stream's structural pass alone (--kernel-mode 50), c2 bench lines
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r04s} && mkdir -p $O && export TMPDIR=/tmp
for m in ${MODES:-0 41 50 51}; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-serve --workload ${WL:-c2} --steps 10 --kernel-mode $m > $O/bench_${WL:-c2}_m$m.log 2>&1 || { echo "bench mode $m failed"; tail -30 $O/bench_${WL:-c2}_m$m.log; exit 1; }
  grep '"metric"' $O/bench_${WL:-c2}_m$m.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d.get('roofline', {})
print('mode $m', d['config'].get('workload'), 'ms', d.get('ms_per_step'), 'kernel_ms', r.get('kernel_ms'), 'frac', r.get('frac'), 'parity', d.get('parity'), 'exact', d.get('exact_path_requests'), 'undecided', d.get('undecided'))"
done
