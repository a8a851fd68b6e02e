# round 5: 2-stage halo conv ring -- tests, microbench, C2 bench
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5n2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_kernels.py > $O/t_k.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_model.py tests/test_gpu_replay.py > $O/t_m.txt 2>&1
timeout -k 10 200 python -u tools/ring_ab.py --only bnb --configs halo,halo-ws --reps 20 --rounds 3 > $O/bnb.txt 2>&1
for i in 1 2 3; do timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/b$i.json 2>/dev/null; grep -o 'ms_per_step": [0-9.]*' $O/b$i.json >> $O/ab.txt; done
cat $O/ab.txt
