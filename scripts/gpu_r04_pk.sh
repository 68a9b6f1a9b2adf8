# round 4: bench lines after the register packing (c2, c3, c5), the small batch profile,
# and the c4 line with the serving leg
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04k} && mkdir -p $O && export TMPDIR=/tmp
line() { grep '"metric"' $1 | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d.get('roofline', {}); sv = d.get('serving') or []
print('$2', 'ms', round(d.get('ms_per_step'), 4), 'kernel_ms', round(r.get('kernel_ms'), 4), 'frac', round(r.get('frac'), 4), 'exact', d.get('exact_path_requests'), 'parity', d.get('parity'))
for s in sv: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')), s.get('batches'))"; }
for wl in c2 c3 c5; do
  timeout -k 10 400 python -u bench.py --no-cpu --no-pcie --no-serve --workload $wl --steps 10 > $O/${wl}.log 2>&1 || { echo "$wl failed"; tail -5 $O/${wl}.log; exit 1; }
  line $O/${wl}.log "$wl"
done
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_n64 -o n64 -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --n 64 --steps 50 > $R/$O/prof_n64.log 2>&1) || { echo "prof n64 failed"; tail -5 $O/prof_n64.log; exit 1; }
python3 - $O/prof_n64 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("  %-60s calls %6s avg_us %8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
timeout -k 10 600 python -u bench.py --no-cpu --no-pcie --workload c4 --steps 5 > $O/c4.log 2>&1 || { echo "c4 failed"; tail -20 $O/c4.log; exit 1; }
line $O/c4.log "c4"
echo done
