export PYTHONPATH=$PWD TMPDIR=/tmp
run() { tag=$1; w=$2; shift 2; timeout -k 10 200 env "$@" python bench.py --steps 20 --warmup $w > gpurun_out/up_$tag.log 2>&1 || { echo "$tag FAILED"; tail -3 gpurun_out/up_$tag.log; exit 1; }; echo "$tag $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/up_$tag.log)"; }
for r in 1 2 3; do run up$r 5 MDA_GRAPH_UPLOAD=1; run noup$r 5 MDA_GRAPH_UPLOAD=0; done
run w30 30 MDA_GRAPH_UPLOAD=1
run w100 100 MDA_GRAPH_UPLOAD=1
