# Steady-state kernel profile of bench.py on a given config: CFG=<yaml> [BATCH=N] [TOP=N] [TAG=name]
set -x
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
name=${TAG:-$(basename ${CFG} .yaml)}
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_$name -o run -- python bench.py --cfg ${CFG} --batch ${BATCH:-64} --steps 20 --warmup 10 ${EXTRA} > gpurun_out/prof_$name.log 2>&1 || { tail -20 gpurun_out/prof_$name.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_$name/run_results.db --skip 12 --top ${TOP:-30} --md gpurun_out/prof_${name}_summary.md | cut -c1-160
python scripts/step_timeline.py gpurun_out/prof_$name/run_results.db > gpurun_out/prof_${name}_timeline.txt
rm -f gpurun_out/prof_$name/run_results.db
