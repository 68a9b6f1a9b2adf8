# round 6: one change under test: the GPU parity file, bench lines (BENCH_WLS), WRITE_SIZE of
# the bench kernels (PMC_WLS), then the serving modes (SERVE_MODES)
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r06t} && mkdir -p $O && export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py} -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -10
[ $rc -eq 0 ] || exit 1
fi
for wl in $BENCH_WLS; do
  timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 3 --cpu-seconds 3 --no-pcie --no-serve > $O/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail -20 $O/bench_$wl.log; exit 1; }
  tail -1 $O/bench_$wl.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$wl', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), d.get('parity'))"
done
for wl in $PMC_WLS; do
  (cd /tmp && timeout -s KILL 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $R/$O/pmc_WRITE_SIZE_$wl -o run -- python3 $R/bench.py --no-cpu --no-pcie --no-serve --workload $wl --steps 2 --warmup 1 > $R/$O/pmc_WRITE_SIZE_$wl.log 2>&1) || { echo "pmc $wl failed"; exit 1; }
  python3 scripts/pmc_summary.py $O/pmc_WRITE_SIZE_$wl 2>&1 | grep -E "scan_lean|unpermute|tenant" | head -5
done
if [ -n "$SERVE_MODES" ]; then
  timeout -k 10 400 python -u scripts/serve_modes.py $SERVE_MODES > $O/serve.log 2>&1 || { echo "serve failed"; tail $O/serve.log; exit 1; }
  grep '"modes"' $O/serve.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['modes'], d['producers'], d['window_us'], 'p50', d['p50_us'], 'p99', d['p99_us'], 'dps', d['decisions_per_s'], 'rpb', d['req_per_batch'], d['equal'], 'wait', d['wait_us'], 'eval', d['eval_us'], 'wake', d['wake_us'], 'resume', d['resume_us'], 'sync', d['sync_us'])"
fi
echo done
