# round 4: c4 serving leg unprofiled (FIN in-kernel finish), then its HIP API trace
R=$GRAFT_REPO_ROOT; cd $R && O=gpurun_out/${OUT:-r04fin2} && mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python3 -u bench.py --no-cpu --no-pcie --workload c4 --n 65536 --steps 5 --warmup 2 > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 1; }
grep '"metric"' $O/bench_c4.log | python3 -c "
import sys, json
d = json.loads(sys.stdin.read())
for s in d.get('serving') or []: print('   serving', s.get('producer_threads'), s.get('window_us'), s.get('latency_us'), round(s.get('decisions_per_s')), s.get('batches'), s.get('equal_to_batch_results'))"
OUT=${OUT:-r04fin2} bash scripts/gpu_r04_serve.sh
