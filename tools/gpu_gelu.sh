set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gelu; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_metaformer.py tests/test_variants.py tests/test_gpu_fullsize.py -m gpu > $O/t.log 2>&1 || { tail -40 $O/t.log; exit 1; }
tail -2 $O/t.log
for m in MetaConv MetaPool; do
timeout -k 10 300 python -u bench.py --model $m --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$m.json 2>$O/bench_$m.err || { tail $O/bench_$m.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_$m.json')); print('$m', d['ms_per_step'], d['value'], d.get('step_mfma_frac'))"
done
