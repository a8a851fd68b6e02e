set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r3p_bench.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/host_time.py --steps 20 > gpurun_out/r3p_host.log 2>&1 || exit 1
bash tools/gpu_prof.sh r3p_prof
