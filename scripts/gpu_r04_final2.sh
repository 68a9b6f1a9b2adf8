# round 4 evidence, part 2: the GPU suite, the bench lines c2..c5 (CPU baseline, parity,
# c4 serving), rocprofv3 stats of each and of a 64-request batch, smoke
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04final2} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20 || true
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
for w in ${WLS:-c2 c3 c4 c5}; do
  timeout -k 10 500 python -u bench.py --workload $w > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$w -o $w -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 5 > $R/$O/prof_$w.log 2>&1) || echo "rocprof $w failed"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_n64 -o n64 -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --n 64 --steps 50 > $R/$O/prof_n64.log 2>&1) || echo "rocprof n64 failed"
grep -h '"metric"' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'].get('workload'), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],4), d['roofline'].get('traffic'), d.get('parity'), d.get('exact_path_requests'), d.get('undecided'), (d.get('cpu_baseline') or {}).get('value'))
    for s in d.get('serving') or []: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok || echo smoke failed
echo done
