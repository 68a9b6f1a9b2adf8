# round 3: c2 step time of variant builds (scripts/var/libauthjx_<v>.so) vs the tree's build
cd $GRAFT_REPO_ROOT && O=gpurun_out/${OUT:-r03j} && mkdir -p $O && export TMPDIR=/tmp
W=${W:-c2}
for v in ${VARS:-v1 hyb v1nob hybnob} full; do
  L=scripts/var/libauthjx_$v.so; [ $v = full ] && L=authorino_amd/libauthjx.so
  AUTHJX_LIB=$L timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --no-serve --workload $W --steps 10 $BARGS > $O/var_${W}_$v.log 2>&1 || { echo "$v failed"; tail -5 $O/var_${W}_$v.log; exit 1; }
  python3 -c "
import json
for l in open('$O/var_${W}_$v.log'):
    if l.startswith('{'): d=json.loads(l); print('$v', round(d['ms_per_step'],3), 'ms', round(d['roofline']['kernel_ms'],3), d.get('mismatches', d.get('parity')))"
done
