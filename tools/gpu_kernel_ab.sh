#!/bin/bash
# GPU-box script: per-kernel time of one kernel family under kernel-library variants, in the step
# (rocprofv3 kernel trace of bench.py, 2 warmup + 5 timed steps per variant; kernel-trace only).
#   KERNEL=stem_bwd_reduce LIBS="- variants/libpda_kernels_X.so" bash tools/gpu_kernel_ab.sh
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/kab
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in $(seq ${REPS:-1}); do
  for lib in ${LIBS:--}; do
    tag=$(echo "$lib" | tr -c 'A-Za-z0-9.\n' '_').$rep
    if [ "$lib" = "-" ]; then unset PDA_KERNEL_LIB; else export PDA_KERNEL_LIB=$lib; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/$tag -o run -- \
      python3 $R/bench.py --steps 5 --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 --util-steps 0 \
      > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
    python3 - "$O/$tag" "${KERNEL}" "$lib" <<'PY'
import csv, glob, statistics, sys
d, k, lib = sys.argv[1:4]
f = glob.glob(f"{d}/**/run_kernel_trace.csv", recursive=True)[0]
t = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(f))
     if k in r["Kernel_Name"]]
print(f"{lib}: {k} n={len(t)} median {statistics.median(t):.1f} us, mean {statistics.mean(t):.1f} us")
PY
  done
done
