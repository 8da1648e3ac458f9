# A/B of hipGraph execution knobs on the flagship bench (teacher/student branch overlap).
set -x
mkdir -p gpurun_out/ab
run() { name=$1; shift; timeout -k 10 200 env "$@" python bench.py --steps 200 --warmup 30 $BENCH_ARGS > gpurun_out/ab/$name.log 2>&1 || { tail -20 gpurun_out/ab/$name.log; return 1; }; echo "$name $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/$name.log)"; }
run default X=1 &&
run nopacket DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
run q4 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 &&
run nopacket_q4 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 DEBUG_HIP_FORCE_GRAPH_QUEUES=4 &&
BENCH_ARGS=--no-graph run nograph X=1 &&
BENCH_ARGS=--no-teacher-stream run noteastream X=1 &&
BENCH_ARGS=--no-teacher-stream run noteastream_nopacket DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 &&
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null &&
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_nopacket -o run -- python bench.py --steps 20 --warmup 10 > gpurun_out/prof_nopacket.log 2>&1 &&
python scripts/step_timeline.py gpurun_out/prof_nopacket/run_results.db > gpurun_out/ab/timeline_nopacket.txt && tail -3 gpurun_out/ab/timeline_nopacket.txt
