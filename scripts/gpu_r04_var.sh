# round 4: kernel durations of a small batch on the default (streaming) path, then lean
# register-budget variants (3 / 2 waves per SIMD, 512-thread groups) on c2 and c3
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04v} && mkdir -p $O && export TMPDIR=/tmp
line() { grep '"metric"' $1 | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d.get('roofline', {})
print('$2', 'ms', round(d.get('ms_per_step'), 4), 'kernel_ms', round(r.get('kernel_ms'), 4), 'frac', round(r.get('frac'), 4), 'exact', d.get('exact_path_requests'))"; }
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_n64 -o n64 -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --n 64 --steps 50 > $R/$O/prof_n64.log 2>&1) || { echo "prof n64 failed"; tail -5 $O/prof_n64.log; exit 1; }
python3 - $O/prof_n64 <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("  %-60s calls %6s avg_us %8.2f" % (r["Name"][:60], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
for wl in c2 c3; do for v in default l3 l2; do
  if [ $v = default ]; then L=""; else L="AUTHJX_LIB=$R/scripts/var/libauthjx_$v.so"; fi
  env $L timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-serve --workload $wl --steps 10 > $O/${wl}_$v.log 2>&1 || { echo "$wl $v failed"; tail -5 $O/${wl}_$v.log; exit 1; }
  line $O/${wl}_$v.log "$wl $v"
done; done
echo done
