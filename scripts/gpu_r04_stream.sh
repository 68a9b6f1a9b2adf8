# round 4: the streaming kernel (default) vs the lean kernel (--kernel-mode 41), the stream's
# structural pass alone (50) and without its fold (51); bench lines per workload
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r04s} && mkdir -p $O && export TMPDIR=/tmp
for wl in ${WLS:-c2}; do
for m in ${MODES:-0 41 50 51}; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-serve --workload $wl --steps 10 --kernel-mode $m > $O/bench_${wl}_m$m.log 2>&1 || { echo "bench $wl mode $m failed"; tail -30 $O/bench_${wl}_m$m.log; exit 1; }
  grep '"metric"' $O/bench_${wl}_m$m.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d.get('roofline', {})
print('mode $m', d['config'].get('workload'), 'ms', round(d.get('ms_per_step'), 4), 'kernel_ms', round(r.get('kernel_ms'), 4), 'frac', round(r.get('frac'), 4), 'parity', d.get('parity'), 'exact', d.get('exact_path_requests'), 'undecided', d.get('undecided'))"
done
done
