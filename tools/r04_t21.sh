# the bench's own N-rank path rehearsed on the one-GPU box (gloo; ranks share the GPU): N = 2, 4
set -o pipefail
for n in 2 4; do
  FISDF_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 2 --warmup 1 > gpurun_out/r04_t21_n$n.json 2> gpurun_out/r04_t21_n$n.err || { echo FAIL $n; tail -20 gpurun_out/r04_t21_n$n.err; exit 1; }
  tail -c 400 gpurun_out/r04_t21_n$n.json; echo
done
exit 0
