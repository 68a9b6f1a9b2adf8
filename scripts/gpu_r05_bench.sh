# round 5: bench lines (c2 tiled and all-unique, c3, c4, c5) on the current tree
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r05bench} && mkdir -p $O && export TMPDIR=/tmp
for spec in ${SPECS:-"c2" "c2 --unique 1048576 --no-cpu --no-pcie" "c3 --no-pcie" "c4" "c5"}; do
  set -- $spec; wl=$1; shift; tag=$wl$(echo "$*" | tr -dc 'a-z0-9' | head -c 12)
  timeout -k 10 500 python -u bench.py --workload $wl "$@" > $O/bench_$tag.log 2>&1 || { echo "bench $spec failed"; tail -20 $O/bench_$tag.log; exit 1; }
  grep '"metric"' $O/bench_$tag.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print('$spec', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],4), d.get('parity'), d.get('exact_path_requests'), d.get('undecided'), (d.get('cpu_baseline') or {}).get('value'))
    for s in d.get('serving') or []: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')), s.get('equal_to_batch_results'))"
done
echo done
