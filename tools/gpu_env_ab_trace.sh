#!/bin/bash
# GPU-box script: kernel tests under a variant library (LIB, optional), an alternating step A/B over
# env variants (VARIANTS, REPS), then one kernel trace per variant with the per-family times of the
# kernels named in FAMILIES (regex) -> gpurun_out/envab/.
set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/envab; mkdir -p $O
[ -n "$LIB" ] && export PDA_KERNEL_LIB=$LIB
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
REPS=${REPS:-3} TAG=envab_ VARIANTS="$VARIANTS" bash tools/gpu_ab_env.sh || exit 1
for v in $VARIANTS; do
  envs=(); [ "$v" != "-" ] && IFS=, read -ra envs <<< "$v"
  tag=$(echo "$v" | tr -c 'A-Za-z0-9.\n' '_')
  (cd /tmp && export TMPDIR=/tmp && for e in "${envs[@]}"; do export "$e"; done && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr_$tag -o run -- python3 $R/bench.py --steps 5 --warmup 2 --fp32-steps 0 --amp-steps 0 --dp-steps 0 > $O/tr_$tag.json 2> $O/tr_$tag.err) || { tail -20 $O/tr_$tag.err; exit 1; }
  python - "$O/tr_$tag" "${FAMILIES:-stem}" "$v" <<'PY'
import csv, glob, re, statistics, sys
sys.path.insert(0, "tools")
from prof_summary import family
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = {}
for r in csv.DictReader(open(f)):
    k = family(r["Kernel_Name"])
    if re.search(sys.argv[2], k):
        d.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
print(sys.argv[3], {k: round(statistics.median(v), 1) for k, v in sorted(d.items())})
PY
done
