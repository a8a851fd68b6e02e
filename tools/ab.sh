# interleaved A/B of the C2 bench on one box: tools/ab.sh "ENV_A" "ENV_B" [rounds]
# (ENV_X: space-separated VAR=value settings, "" for the default); prints ms/step per run
set -o pipefail
cd $GRAFT_REPO_ROOT
A="$1"; B="$2"; N=${3:-3}
for i in $(seq 1 $N); do
  for tag in A B; do
    if [ $tag = A ]; then E="$A"; else E="$B"; fi
    env $E timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-kernel-timing > gpurun_out/ab_$tag$i.log 2>&1 || exit 1
    echo "$tag [$E] $(grep -ho '"ms_per_step": [0-9.]*' gpurun_out/ab_$tag$i.log)" | tee -a gpurun_out/ab.txt
  done
done
