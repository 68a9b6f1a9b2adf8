# round 4: the lean walker with its rare fields packed (spills): parity, c2 / c3 times, scratch
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04pack}/pack && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for wl in c2 c3; do
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$wl -o run -- python3 $R/bench.py --no-cpu --no-serve --workload $wl --steps 20 --warmup 3 > $R/$O/bench_$wl.log 2>&1) || { echo "bench $wl failed"; tail -5 $O/bench_$wl.log; exit 1; }
  python3 - $O/prof_$wl $wl <<'PY'
import csv, glob, sys, json
d = sys.argv[1]
for f in glob.glob(d + "/**/*kernel_stats.csv", recursive=True):
    for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:3]:
        print("  %s %-50s calls %5s avg_us %8.2f" % (sys.argv[2], r["Name"][:50], r["Calls"], float(r["AverageNs"]) / 1e3))
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    seen = set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        if "lean" in k and k not in seen:
            seen.add(k)
            print("  %s %s scratch %s vgpr %s sgpr %s" % (sys.argv[2], k, r["Scratch_Size"], r["VGPR_Count"], r["SGPR_Count"]))
PY
  grep '"metric"' $O/bench_$wl.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('  bench', d['config']['workload'], 'ms', round(d['ms_per_step'],4), 'frac', d['roofline']['frac'], 'parity', d.get('parity',{}).get('mismatches') if isinstance(d.get('parity'),dict) else d.get('parity'))"
done
echo done
