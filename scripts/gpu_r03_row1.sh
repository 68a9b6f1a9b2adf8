# round 3, first GPU pass of the row kernel: GPU suite, then c2..c5 bench lines (row
# kernel default vs the token-scanner kernel, --kernel-mode 40), then rocprofv3 stats
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r03a && export TMPDIR=/tmp
O=gpurun_out/r03a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "GPU tests failed rc=$?"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for w in c2 c3 c5; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  timeout -k 10 240 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 --kernel-mode 40 > $O/bench_${w}_old.log 2>&1 || { echo "bench old $w failed"; exit 1; }
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pcie --workload c2 --steps 5 > $GRAFT_REPO_ROOT/$O/prof_c2.log 2>&1 || echo "rocprof failed"
cd $GRAFT_REPO_ROOT && grep -h '"metric"' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'].get('workload'), d.get('ms_per_step'), d.get('roofline',{}).get('frac'), d.get('parity'))"
