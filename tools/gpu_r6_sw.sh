export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1; mkdir -p gpurun_out/sw
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/sw/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/sw/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/conv_bench.py 400 3 > gpurun_out/sw/conv_bench.txt 2>&1 || { tail -20 gpurun_out/sw/conv_bench.txt; exit 1; }
REPS=3 TAG=sw_ VARIANTS="PDA_KERNEL_LIB=ab/libpda_kernels_prev.so -" bash tools/gpu_ab_env.sh || exit 1
O=gpurun_out/dprep; mkdir -p $O; R=$(pwd); cd /tmp && export TMPDIR=/tmp; PDA_DP_FORCE_REPLAY=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/bench.py --dp --gpus 1 --steps 5 --warmup 3 > $R/$O/bench.json 2> $R/$O/bench.err || { tail -20 $R/$O/bench.err; exit 1; }
cd $R; python tools/prof_summary.py $O/prof 16 > $O/prof_summary.md; python tools/stream_timeline.py $O/prof > $O/timeline.txt; python tools/step_sequence.py $O/prof > $O/seq.txt; cat $O/timeline.txt; tail -3 $O/seq.txt
