set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_disc.py -k "persistent_backward or early_slice" > gpurun_out/r3d_tests.log 2>&1 || exit 1
for cfg in "0 0" "0 8" "0 32" "1 0" "1 2" "1 8"; do
  set -- $cfg
  echo "=== SAMPLE=$1 NAP=$2" >> gpurun_out/r3d_forms.log
  AVC_LSTM_SAMPLE=$1 AVC_LSTM_NAP=$2 HS=1024 FORMS=3,2 timeout -k 10 200 python -u tools/lstm_bwd_forms.py 1 >> gpurun_out/r3d_forms.log 2>&1 || exit 1
done
