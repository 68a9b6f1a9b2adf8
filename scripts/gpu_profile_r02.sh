# round-2 evidence: GPU parity, per-workload kernel stats (rocprofv3 --kernel-trace
# --stats, csv), FETCH_SIZE / WRITE_SIZE passes (one counter group per run), bench lines
cd $GRAFT_REPO_ROOT && O=gpurun_out/r02 && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
for w in c2 c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o $w -- python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > $O/prof_$w.log 2>&1 || exit $?
done
for w in c2 c3 c4 c5; do
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$w -o f -- python -u bench.py --no-cpu --no-pcie --workload $w --steps 2 --warmup 1 > $O/pmc_fetch_$w.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$w -o w -- python -u bench.py --no-cpu --no-pcie --workload $w --steps 2 --warmup 1 > $O/pmc_write_$w.log 2>&1 || exit $?
done
