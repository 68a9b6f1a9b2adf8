# round 3: where the row kernel's time goes (c2): P1 only (42), P1+P2 (43), + captures
# (44), the full row kernel (41, no exact pass), the default step (0), token kernel (40)
cd $GRAFT_REPO_ROOT && O=gpurun_out/r03e && mkdir -p $O && export TMPDIR=/tmp
for m in 42 43 44 41 0 40; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload ${W:-c2} --steps 10 --kernel-mode $m > $O/abl_${W:-c2}_$m.log 2>&1 || { echo "mode $m failed"; tail -5 $O/abl_${W:-c2}_$m.log; exit 1; }
  python3 -c "
import json,sys
for l in open('$O/abl_${W:-c2}_$m.log'):
    if l.startswith('{'): d=json.loads(l); print('mode $m', round(d['ms_per_step'],3), 'ms', d['roofline']['kernel_ms'])"
done
