# GEMM microbench across NT-kernel configurations (AVC_NT_CFG = "BN,NST"; "0" = old fast kernel)
set -e
for cfg in 0 128,2 128,3 128,4 64,2 64,3 64,4; do
  echo "== AVC_NT_CFG=$cfg"
  AVC_NT_CFG=$cfg timeout -k 10 120 python tools/gemm_bench.py 2>&1 | grep -v amdgpu.ids | grep -v hipBLASLt
done
