set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fault.py tests/test_gpu_fullsize.py tests/test_gpu_disc.py tests/test_gpu_dist.py -s > gpurun_out/t_new.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1
