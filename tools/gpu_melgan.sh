set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/melgan; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_melgan.py -m gpu > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
grep -E "PASS|FAIL" $O/t.log
timeout -k 10 120 python -u tools/vocoder_bench.py > $O/bench.json 2>$O/bench.err || { cat $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/vocoder_bench.py > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
cut -d, -f1-4 $(find $GRAFT_REPO_ROOT/$O/prof -name "run_kernel_stats.csv") | head -14
