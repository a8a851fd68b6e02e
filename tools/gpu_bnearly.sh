# round 5: forward BN statistics handed over before the C stores -- tests, microbench, C2 / C5 A/B
set -e
export TMPDIR=/tmp
O=gpurun_out/${1:-r5be}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_ring.py tests/test_gpu_kernels.py -k "ring or bn or conv" > $O/t_kernels.txt 2>&1
timeout -k 10 200 python -u tools/ring_ab.py --only c2 --configs halo,auto --reps 20 --rounds 3 > $O/c2.txt 2>&1
timeout -k 10 200 python -u tools/ring_ab.py --only utt --configs halo --reps 20 --rounds 3 > $O/utt.txt 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_capture.py tests/test_gpu_model.py tests/test_gpu_metaformer.py > $O/t_model.txt 2>&1
for i in 1 2; do timeout -k 10 120 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/b$i.json 2>/dev/null; grep -o 'ms_per_step": [0-9.]*' $O/b$i.json >> $O/ab.txt; done
cat $O/ab.txt
