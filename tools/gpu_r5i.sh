set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r5i
timeout -k 10 300 python tools/halo_bench.py 20 2>&1 | tee gpurun_out/r5i/halo.txt || exit 1
# graph-queue reproducer (tools/graph_queue_repro.py): single queue first, then HIP's default
for a in "1 --side --threads 2" "0" "0 --side" "0 --side --threads 2" "0 --side --threads 4 --segments 8"; do
  set -- $a; q=$1; shift
  echo "== DEBUG_HIP_FORCE_GRAPH_QUEUES=$q $*" | tee -a gpurun_out/r5i/repro.txt
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 120 python tools/graph_queue_repro.py "$@" >> gpurun_out/r5i/repro.txt 2>&1
  rc=$?; echo "rc=$rc" | tee -a gpurun_out/r5i/repro.txt
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r5i/repro.txt; exit 0; }
done
tail -12 gpurun_out/r5i/repro.txt
