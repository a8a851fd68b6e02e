set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_metaformer.py tests/test_variants.py -m gpu > gpurun_out/t_mf.log 2>&1 || { tail -30 gpurun_out/t_mf.log; exit 1; }
tail -1 gpurun_out/t_mf.log
echo "== MetaConv"; bash tools/ab_head.sh "--model MetaConv --steps 10 --warmup 3" "" 2 || exit 1
echo "== C2"; bash tools/ab_head.sh "--steps 30 --warmup 5" "" 2 || exit 1
