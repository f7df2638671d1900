set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
O=gpurun_out/r5ad; mkdir -p $O
PDA_DIST_BACKEND=gloo PDA_COMM=torch timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --batch 64 \
  > $O/bench_rehearse2.json 2> $O/bench_rehearse2.err || { tail -30 $O/bench_rehearse2.err; exit 1; }
cat $O/bench_rehearse2.json
