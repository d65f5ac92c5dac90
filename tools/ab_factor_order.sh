set -o pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
for v in 1 0; do
FISDF_FACTOR_AFTER_Y=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/ab/b_${v}_$i.json 2>gpurun_out/ab/e_${v}_$i.log || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab/b_${v}_$i.json')); print('after_y=$v', d['ms_per_step'])"
done; done
