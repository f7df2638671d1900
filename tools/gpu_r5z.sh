set -o pipefail
export PDA_NO_BUILD=1 PYTHONUNBUFFERED=1
PDA_FORK_TRACK=0 STEPS=5 bash tools/gpu_profile.sh > /dev/null || exit 1
mkdir -p gpurun_out/prof_r5 && cp gpurun_out/prof/summary.md gpurun_out/prof_r5/summary_track0.md
python /root/repo/tools/stream_timeline.py gpurun_out/prof > gpurun_out/prof_r5/timeline_track0.txt 2>&1 || true
head -40 gpurun_out/prof_r5/summary_track0.md
