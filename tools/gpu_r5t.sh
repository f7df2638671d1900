set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
R=$(pwd)
mkdir -p gpurun_out/r5t
cd /tmp && export TMPDIR=/tmp
for v in default dk0 dk1; do
  envs=""
  [ $v = dk0 ] && export HIP_FORCE_DEV_KERNARG=0
  [ $v = dk1 ] && export HIP_FORCE_DEV_KERNARG=1
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r5t/$v -o run -- python3 $R/tools/gap_bench.py 60 > $R/gpurun_out/r5t/$v.log 2>&1 || { tail -5 $R/gpurun_out/r5t/$v.log; exit 1; }
  unset HIP_FORCE_DEV_KERNARG
  echo "== $v"; python3 $R/tools/gap_bench.py --summary $R/gpurun_out/r5t/$v
done
