# round 4: where the serving leg's time goes (kernel + HIP API trace of bench.py's c4 leg)
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04s} && mkdir -p $O && export TMPDIR=/tmp
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $R/$O/prof_serve -o serve -- python3 $R/bench.py --no-cpu --no-pcie --workload c4 --n 65536 --steps 2 --warmup 1 > $R/$O/prof_serve.log 2>&1) || { echo "prof failed"; tail -5 $O/prof_serve.log; exit 1; }
python3 - $O/prof_serve <<'PY'
import csv, glob, sys
for pat in ("kernel_stats", "hip_api_stats"):
    for f in glob.glob(sys.argv[1] + "/**/*%s.csv" % pat, recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:14]
        for r in rows:
            print("  %-14s %-58s calls %7s avg_us %9.2f total_ms %9.2f" % (pat[:12], r["Name"][:58], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
grep '"metric"' $O/prof_serve.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
for s in d.get('serving') or []: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')), s.get('batches'))"
echo done
