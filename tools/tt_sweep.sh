# weight-gradient GEMM shapes under each TT kernel configuration (AVC_TT_CFG = "BMT,NST"; 0 = 2-stage)
cd $GRAFT_REPO_ROOT
for cfg in 0 128,2 256,2 256,3; do
  echo "== AVC_TT_CFG=$cfg"
  AVC_TT_CFG=$cfg timeout -k 10 120 python -u tools/tt_bench.py 2>/dev/null || exit 1
done
echo "== halo 3 stages"
AVC_TT_HALO=3 timeout -k 10 120 python -u tools/tt_bench.py 2>/dev/null | head -3
