set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/bnb; mkdir -p $O
timeout -k 10 120 python -u tools/bn_bwd_bench.py > $O/bench.log 2>&1 || { cat $O/bench.log; exit 1; }
grep -v amdgpu $O/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bn_bwd_bench.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cut -d, -f1-4 $(find $GRAFT_REPO_ROOT/$O/prof -name "run_kernel_stats.csv") | head -8
