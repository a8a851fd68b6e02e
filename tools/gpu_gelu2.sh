set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/gelu2; mkdir -p $O
for f in 0 1 2 3; do
AVC_GELU_FUSE=$f timeout -k 10 300 python -u bench.py --model MetaConv --steps 10 --warmup 3 --no-cpu-baseline > $O/b$f.json 2>$O/b$f.err || { tail $O/b$f.err; exit 1; }
python -c "import json; d=json.load(open('$O/b$f.json')); print('FUSE=$f', d['ms_per_step'])"
done
