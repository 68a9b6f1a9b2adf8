# round 4: small-batch latency after the in-kernel stage B, stream tests, c4 serving
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04l2} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
line() { grep '"metric"' $1 | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d.get('roofline', {}); sv = d.get('serving') or []
print('$2', 'ms', round(d.get('ms_per_step'), 4), 'kernel_ms', round(r.get('kernel_ms'), 4), 'frac', round(r.get('frac'), 4), 'exact', d.get('exact_path_requests'))
for s in sv: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')))"; }
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_n64 -o n64 -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --n 64 --steps 50 > $R/$O/prof_n64.log 2>&1) || { echo "prof n64 failed"; tail -5 $O/prof_n64.log; exit 1; }
python3 - $O/prof_n64 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("  %-60s calls %6s avg_us %8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
line $O/prof_n64.log "c2 n=64"
timeout -k 10 600 python -u bench.py --no-cpu --no-pcie --workload c4 --steps 5 > $O/c4.log 2>&1 || { echo "c4 failed"; tail -20 $O/c4.log; exit 1; }
line $O/c4.log "c4 default"
echo done
