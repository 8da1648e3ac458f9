# scratch GPU command file (see scripts/gpu_run.sh for the parameterised runs)
export PYTHONPATH=$PWD TMPDIR=/tmp
BENCH="--steps 300 --warmup 30" bash scripts/gpu_run.sh
