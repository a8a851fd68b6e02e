# MetaConv (C4) bench line + kernel-trace stats and step breakdown
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/mc; mkdir -p $O
timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['value'], d.get('step_mfma_frac'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model MetaConv --steps 5 --warmup 2 --no-cpu-baseline --no-kernel-timing > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || exit 1
python3 $GRAFT_REPO_ROOT/tools/step_breakdown.py $(find $GRAFT_REPO_ROOT/$O/prof -name "run_kernel_trace.csv") 40 > $GRAFT_REPO_ROOT/$O/breakdown.txt
head -70 $GRAFT_REPO_ROOT/$O/breakdown.txt
