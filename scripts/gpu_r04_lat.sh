# round 4: GPU suite with the streaming kernel as the small-batch path, then bench lines:
# c2 at 1M (lean default vs the stream at 32 requests per wave), small batches (stream vs
# lean), and the c4 serving leg (multi-tenant latency batches on the stream)
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04l} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "FAILED|ERROR" $O/pytest.log | head -20
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
line() { grep '"metric"' $1 | python3 -c "
import sys, json
d = json.loads(sys.stdin.read()); r = d.get('roofline', {}); s = d.get('serving') or {}
print('$2', 'ms', round(d.get('ms_per_step'), 4), 'kernel_ms', round(r.get('kernel_ms'), 4), 'frac', round(r.get('frac'), 4), 'parity', d.get('parity'), 'exact', d.get('exact_path_requests'), 'undecided', d.get('undecided'), 'serving', {k: s.get(k) for k in ('p50_us', 'p99_us', 'decisions_per_s')} if s else None)"; }
for m in 0 52; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-serve --workload c2 --steps 10 --kernel-mode $m > $O/c2_m$m.log 2>&1 || { echo "c2 $m failed"; tail -20 $O/c2_m$m.log; exit 1; }
  line $O/c2_m$m.log "c2 mode $m"
done
for n in 64 512 4096; do for m in 0 41; do
  timeout -k 10 300 python -u bench.py --no-cpu --no-pcie --no-serve --workload c2 --n $n --steps 20 --kernel-mode $m > $O/c2_n${n}_m$m.log 2>&1 || { echo "c2 n $n $m failed"; tail -20 $O/c2_n${n}_m$m.log; exit 1; }
  line $O/c2_n${n}_m$m.log "c2 n=$n mode $m"
done; done
timeout -k 10 600 python -u bench.py --no-cpu --no-pcie --workload c4 --steps 5 > $O/c4.log 2>&1 || { echo "c4 failed"; tail -20 $O/c4.log; exit 1; }
line $O/c4.log "c4 default"
echo done
