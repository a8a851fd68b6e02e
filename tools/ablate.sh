# step-time ablations of the C2 bench (diagnostic builds of the path, wrong gradients)
cd $GRAFT_REPO_ROOT
echo "baseline"; timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c150-260
echo "baseline graph"; timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c150-260
echo "no side-stream wgrads"; AVC_ABLATE_WGRAD=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c150-260
echo "no side-stream wgrads, graph"; AVC_ABLATE_WGRAD=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --graph --no-cpu-baseline --no-kernel-timing 2>/dev/null | cut -c150-260
