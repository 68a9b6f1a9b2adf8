# A/B of the single-pass kernel's workgroup size (kernel modes 10/11/12 = 4/8/16 waves)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/blk && export TMPDIR=/tmp
for w in ${WORKLOADS:-c2 c3}; do for m in 0 10 11 12; do
  timeout -k 10 200 python -u bench.py --no-cpu --no-pcie --workload $w --steps 10 --kernel-mode $m > gpurun_out/blk/${w}_m$m.log 2>&1 || exit $?
done; done
