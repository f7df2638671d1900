#!/bin/bash
# RCCL configuration sweep for a multi-GPU MI355X node (channel count vs the 7 xGMI
# links per GPU, protocol, algorithm). For each world size and setting: the collective sweep
# (tools/rccl_bench.py under torchrun: alpha and bus bandwidth) and the DDP step
# (bench.py --gpus N: images/s, exposed_comm_ms, bucket_allreduce_ms). One JSON line per run in
# gpurun_out/rccl_sweep/results.jsonl. Needs >= max(WORLDS) GPUs; each run is time-limited.
#   WORLDS="2 4 8" CHANNELS="0 8 16 32" PROTOS=" LL128 Simple" bash tools/rccl_sweep.sh
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1 HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/rccl_sweep
mkdir -p $O
ngpu=$(python -c "import torch; print(torch.cuda.device_count())")
port=29700
for n in ${WORLDS:-2 4 8}; do
  [ "$n" -gt "$ngpu" ] && { echo "skip world $n: $ngpu GPUs visible"; continue; }
  for ch in ${CHANNELS:-0 8 16 32}; do
    for proto in ${PROTOS:-"" LL128 Simple}; do
      tag="n${n}_ch${ch}_${proto:-auto}"
      env=()
      [ "$ch" != 0 ] && env+=(NCCL_MIN_NCHANNELS=$ch NCCL_MAX_NCHANNELS=$ch)
      [ -n "$proto" ] && env+=(NCCL_PROTO=$proto)
      port=$((port + 1))
      env "${env[@]}" timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $port tools/rccl_bench.py --max-mb 128 --reps 10 \
        > $O/$tag.coll.txt 2>&1 || { echo "FAIL coll $tag"; tail -5 $O/$tag.coll.txt; exit 1; }
      port=$((port + 1))
      ncarg=(); [ "$ch" != 0 ] && ncarg=(--nccl-channels $ch)
      prarg=(); [ -n "$proto" ] && prarg=(--nccl-proto $proto)
      timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $port bench.py --gpus $n --steps 20 --warmup 5 \
        --fp32-steps 0 --amp-steps 0 --dp-steps 0 "${ncarg[@]}" "${prarg[@]}" \
        > $O/$tag.bench.json 2> $O/$tag.bench.err || { echo "FAIL bench $tag"; tail -5 $O/$tag.bench.err; exit 1; }
      python - "$tag" "$O" <<'PY'
import json, sys
tag, o = sys.argv[1], sys.argv[2]
coll = [json.loads(l) for l in open(f"{o}/{tag}.coll.txt") if l.startswith("{")]
b = json.loads([l for l in open(f"{o}/{tag}.bench.json") if l.startswith("{")][-1])
big = [r for r in coll if r.get("bytes") == 128 << 20]
rec = {"tag": tag, "images_per_sec": b["value"], "ms_per_step": b["ms_per_step"],
       "exposed_comm_ms": b.get("exposed_comm_ms"), "bucket_allreduce_ms": b.get("bucket_allreduce_ms"),
       "busbw_128MB_GBs": big[0]["busbw_GBs"] if big else None,
       "alpha_us": next((r["alpha_us"] for r in coll if "alpha_us" in r), None)}
print(json.dumps(rec))
open(f"{o}/results.jsonl", "a").write(json.dumps(rec) + "\n")
PY
    done
  done
done
