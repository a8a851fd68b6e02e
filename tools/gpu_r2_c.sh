set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/small_lstm_bench.py > gpurun_out/small_lstm.log 2>&1
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1
