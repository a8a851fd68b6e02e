# GPU tests, then a same-box A/B of the fused BN-backward statistics (AVC_BNB) on the bench step
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/s5; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 200 python -u tools/aten_ops.py > $OUT/aten_ops.log 2>&1 || { tail -20 $OUT/aten_ops.log; exit 1; }
cat $OUT/aten_ops.log | grep -v amdgpu
bash $R/tools/gpu_envab.sh s5ab "AVC_X=1" "AVC_APPLY8=0" "AVC_BNB=0"
