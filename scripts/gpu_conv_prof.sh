set -x
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt -o run -- python scripts/conv_microbench.py --iters 20 > gpurun_out/kt.log 2>&1 || { tail -20 gpurun_out/kt.log; exit 1; }
python scripts/kernel_times.py gpurun_out/kt/run_results.db "conv" | grep -v naive
python scripts/kernel_times.py gpurun_out/kt/run_results.db "wgrad"
python scripts/kernel_times.py gpurun_out/kt/run_results.db "split"
python scripts/kernel_times.py gpurun_out/kt/run_results.db "ck::" | head -20
python scripts/kernel_times.py gpurun_out/kt/run_results.db "igemm" | head -20
