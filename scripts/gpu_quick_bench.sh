# quick A/B: c2 / c3 bench of the default kernel (no CPU baseline)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qb && export TMPDIR=/tmp
for w in ${WORKLOADS:-c2 c3}; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 > gpurun_out/qb/$w.log 2>&1 || exit $?
done
