# divergence probe: c2 with 1, 64, 1024 and 16384 document templates (same sizes)
cd $GRAFT_REPO_ROOT && O=gpurun_out/uniq && mkdir -p $O && export TMPDIR=/tmp
for u in 1 64 1024 16384; do
  timeout -k 10 300 python bench.py --workload c2 --no-cpu --no-pcie --unique $u > $O/bench_u$u.log 2>&1 || exit $?
done
