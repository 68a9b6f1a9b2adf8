# round 3: row kernel GPU pass (tests, c2/c3/c5 bench row vs token-scanner kernel, rocprofv3 stats)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03b && export TMPDIR=/tmp
O=gpurun_out/r03b
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -5 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
for w in c2 c3 c5; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  timeout -k 10 240 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 --kernel-mode 40 > $O/bench_${w}_old.log 2>&1 || { echo "bench old $w failed"; exit 1; }
done
grep -h '"metric"' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'].get('workload'), d.get('ms_per_step'), d['roofline'].get('kernel_ms'), d.get('roofline',{}).get('frac'), d.get('exact_path_requests'), d.get('undecided'))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pcie --workload c2 --steps 5 > $GRAFT_REPO_ROOT/$O/prof_c2.log 2>&1 || echo "rocprof failed"
