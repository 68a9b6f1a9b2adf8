# round-2 baseline of the round-1 kernel on unique documents: bench c2 + rocprofv3 kernel stats
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r02base && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --no-pcie > gpurun_out/r02base/bench_c2.log 2>&1 || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02base/prof -o c2 -- python -u bench.py --no-cpu --no-pcie --steps 10 > gpurun_out/r02base/prof_c2.log 2>&1 || exit $?
