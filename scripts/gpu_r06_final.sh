# round 6 evidence on the final tree: the GPU suite; FETCH_SIZE / WRITE_SIZE passes (one
# counter per pass) of c2..c5 and the loads-only calibration (the ablation build), summarised
# on the box into pmc_traffic.json (commit $AJX_COMMIT) before the bench lines, so that every
# line's roofline.traffic is this tree's; bench lines c2 (tiled, all-unique), c3, c4, c5 and
# rocprofv3 --kernel-trace --stats of each; the SQ instruction mix of the lean kernel's
# stage-A ablations (c2, c3); the load-shape micro-benchmark; smoke
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r06final} && mkdir -p $O && export TMPDIR=/tmp
export AJX_COMMIT=${AJX_COMMIT:-unknown}
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20 || true
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
fi
if [ -z "$NOPMC" ]; then
for wl in ${PMC_WLS:-c2 c3 c4 c5}; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $R/$O/pmc_${c}_$wl -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $wl --steps 2 --warmup 1 > $R/$O/pmc_${c}_$wl.log 2>&1) || { echo "pmc $c $wl failed"; exit 1; }
  done
done
(cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_cal -o run -- python3 $R/scripts/prof_modes.py --workload c2 --modes 15 --reps 2 --lib $R/scripts/var/libauthjx_abl.so > $R/$O/pmc_cal.log 2>&1) || { echo "pmc cal failed"; exit 1; }
cp pmc_traffic.json $O/pmc_traffic_before.json
timeout -k 10 300 python3 scripts/fetch_calibration.py $O/pmc_cal c2 1048576 pmc_traffic.json "ajx_scan_lean<true, 1, " > $O/pmc_summary.log 2>&1 || { echo "calibration failed"; tail $O/pmc_summary.log; exit 1; }
for wl in ${PMC_WLS:-c2 c3 c4 c5}; do
  n=1048576; k=ajx_scan_lean; [ $wl = c4 ] && { n=2097152; k=ajx_scan_fused_tenant; }; [ $wl = c5 ] && n=2097152
  python3 scripts/pmc_traffic.py $O/pmc_FETCH_SIZE_$wl $O/pmc_WRITE_SIZE_$wl $wl $n pmc_traffic.json $k >> $O/pmc_summary.log 2>&1 || { echo "pmc summary $wl failed"; exit 1; }
done
cp pmc_traffic.json $O/pmc_traffic.json
fi
for spec in ${SPECS:-c2 c2u c3 c4 c5}; do
  wl=${spec%u}; extra=""; [ "$spec" != "$wl" ] && extra="--unique 1048576"
  timeout -k 10 500 python -u bench.py --workload $wl $extra > $O/bench_$spec.log 2>&1 || { echo "bench $spec failed"; tail -20 $O/bench_$spec.log; exit 1; }
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$spec -o $spec -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $wl $extra --steps 5 > $R/$O/prof_$spec.log 2>&1) || { echo "rocprof $spec failed"; exit 1; }
done
if [ -z "$NOSQ" ]; then
for wl in c2 c3; do
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d $R/$O/sq_$wl -o run -- python3 $R/scripts/prof_modes.py --workload $wl --modes 0,15,16,17,18 --reps 2 --lib $R/scripts/var/libauthjx_abl.so > $R/$O/sq_$wl.log 2>&1) || { echo "sq $wl failed"; exit 1; }
  timeout -k 10 200 python -u scripts/prof_modes.py --workload $wl --modes 0,15,16,17,18,0 --reps 5 --lib scripts/var/libauthjx_abl.so > $O/time_$wl.log 2>&1 || { echo "time $wl failed"; exit 1; }
done
fi
[ -x scripts/var/ubench_loads ] && (timeout -k 10 120 scripts/var/ubench_loads > $O/ubench_loads.txt 2>&1 || echo "ubench failed")
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && echo smoke ok || echo smoke failed
grep -h '"metric"' $O/bench_*.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); c = d['config']; r = d['roofline']; print(c.get('workload'), c.get('unique_templates'), round(d['ms_per_step'],3), round(r['kernel_ms'],3), round(r['frac'],4), r.get('traffic'), (r.get('traffic_source') or {}).get('commit'), d.get('parity'), d.get('exact_path_requests'), d.get('undecided'))"
echo done
