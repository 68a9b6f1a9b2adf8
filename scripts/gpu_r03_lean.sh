# round 3: the lean single-pass kernel (default) vs the token scanner (--kernel-mode 40):
# GPU suite, c2/c3/c5 bench lines, rocprofv3 stats of c2
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r03f} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20 || true
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
for w in c2 c3 c5; do
  timeout -k 10 240 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  timeout -k 10 240 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 --kernel-mode 40 > $O/bench_${w}_old.log 2>&1 || { echo "bench old $w failed"; exit 1; }
done
grep -h '"metric"' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'].get('workload'), d.get('ms_per_step'), d['roofline'].get('kernel_ms'), d['roofline'].get('frac'), d.get('parity'), d.get('exact_path_requests'), d.get('undecided'))"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --no-pcie --workload c2 --steps 5 > $GRAFT_REPO_ROOT/$O/prof_c2.log 2>&1 || echo "rocprof failed"
