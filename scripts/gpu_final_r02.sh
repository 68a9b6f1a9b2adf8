# round-2 evidence on the committed tree: GPU parity, smoke, per-workload kernel stats
# (rocprofv3 --kernel-trace --stats), FETCH_SIZE / WRITE_SIZE passes (one counter per run)
# merged into pmc_traffic.json, then the bench lines (with the CPU baseline) that read it
cd $GRAFT_REPO_ROOT && O=gpurun_out/r02f && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
for w in c2 c3 c4 c5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats_$w -o $w -- python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > $O/prof_$w.log 2>&1 || exit $?
done
rm -f $O/pmc_traffic.json
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_calib -o f -- python -u bench.py --no-cpu --no-pcie --workload c2 --kernel-mode 1 --steps 2 --warmup 1 > $O/pmc_fetch_calib.log 2>&1 || exit $?
python scripts/fetch_calibration.py $O/pmc_fetch_calib c2 1048576 $O/pmc_traffic.json > $O/fetch_calibration.log 2>&1 || exit $?
for w in c2 c3 c4 c5; do
  n=1048576; [ $w = c4 ] && n=2097152; [ $w = c5 ] && n=2097152
  timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$w -o f -- python -u bench.py --no-cpu --no-pcie --workload $w --steps 2 --warmup 1 > $O/pmc_fetch_$w.log 2>&1 || exit $?
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$w -o w -- python -u bench.py --no-cpu --no-pcie --workload $w --steps 2 --warmup 1 > $O/pmc_write_$w.log 2>&1 || exit $?
  python scripts/pmc_traffic.py $O/pmc_fetch_$w $O/pmc_write_$w $w $n $O/pmc_traffic.json > $O/pmc_traffic_$w.log 2>&1 || exit $?
done
cp $O/pmc_traffic.json pmc_traffic.json
for w in c2 c3 c4 c5; do
  timeout -k 10 600 python -u bench.py --workload $w > $O/bench_$w.log 2>&1 || exit $?
done
echo ok > $O/done
