# 256-row conv tiles (AVC_CONV_CFG=13,32,64): parity, isolated timing, step A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/${1:-r3s9}
mkdir -p $OUT
AVC_CONV_CFG=13,32,64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "conv or gemm_bn or fold or window_and_bn" > $OUT/tests13.log 2>&1 || { tail -30 $OUT/tests13.log; exit 1; }
tail -2 $OUT/tests13.log
timeout -k 10 120 python -u tools/conv_ab.py > $OUT/conv_ab.log 2>&1 || exit 1
AVC_CONV_CFG=13,32,64 timeout -k 10 120 python -u tools/conv_ab.py >> $OUT/conv_ab.log 2>&1 || exit 1
cat $OUT/conv_ab.log | grep -v amdgpu
for r in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_def.log || exit 1
AVC_CONV_CFG=13,32,64 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 >> $OUT/bench_13.log || exit 1
done
