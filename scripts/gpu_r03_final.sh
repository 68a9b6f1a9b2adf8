# round 3 evidence on the final tree: HBM traffic passes (FETCH_SIZE / WRITE_SIZE, one
# counter per pass) of the dominant kernel per workload -> pmc_traffic.json, the SQ mix of
# c2, the GPU suite, the bench lines c2..c5 (CPU baseline, parity), rocprofv3 stats, smoke
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r03final} && mkdir -p $O && export TMPDIR=/tmp
ns() { case $1 in c4|c5) echo 2097152;; *) echo 1048576;; esac; }
for w in ${WLS:-c2 c3 c4 c5}; do
  k=ajx_scan_lean; [ $w = c4 ] && k=ajx_scan_fused_tenant
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_f_$w -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 2 --warmup 1 > $R/$O/pmc_f_$w.log 2>&1) || { echo "pmc fetch $w failed"; exit 1; }
  (cd /tmp && timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_w_$w -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 2 --warmup 1 > $R/$O/pmc_w_$w.log 2>&1) || { echo "pmc write $w failed"; exit 1; }
  python3 scripts/pmc_traffic.py $O/pmc_f_$w $O/pmc_w_$w $w $(ns $w) pmc_traffic.json $k > $O/pmc_$w.txt || exit 1
done
(cd /tmp && timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/pmc_sq_c2 -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload c2 --steps 2 --warmup 1 > $R/$O/pmc_sq_c2.log 2>&1) || { echo "pmc sq failed"; exit 1; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20 || true
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
for w in c2 c3 c4 c5; do
  timeout -k 10 400 python -u bench.py --workload $w > $O/bench_$w.log 2>&1 || { echo "bench $w failed"; tail -20 $O/bench_$w.log; exit 1; }
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$w -o $w -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $w --steps 5 > $R/$O/prof_$w.log 2>&1) || echo "rocprof $w failed"
done
grep -h '"metric"' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['config'].get('workload'), round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['roofline']['frac'],4), d['roofline'].get('traffic'), d.get('parity'), d.get('exact_path_requests'), d.get('undecided'), (d.get('cpu_baseline') or {}).get('value'))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok || echo smoke failed
cp pmc_traffic.json $O/pmc_traffic.json
