# round 4: small-batch phase clocks, stream GPU tests and the c4 serving leg
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04ph2} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/lat_phases.py > $O/phases.log 2>&1 || { tail -5 $O/phases.log; exit 1; }
tail -2 $O/phases.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_parity.py -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_serve -o serve -- python3 $R/bench.py --no-cpu --no-pcie --workload c4 --n 65536 --steps 2 --warmup 1 > $R/$O/prof_serve.log 2>&1) || { echo "prof failed"; tail -5 $O/prof_serve.log; exit 1; }
python3 - $O/prof_serve <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:6]:
        print("  %-60s calls %6s avg_us %8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
grep '"metric"' $O/prof_serve.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
for s in d.get('serving') or []: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')), s.get('batches'))"
echo done
