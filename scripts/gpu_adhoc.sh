export TMPDIR=/tmp
run() {  # label, dir, env...
  local label=$1 dir=$2; shift 2
  echo "== $label" | tee -a gpurun_out/ab3.txt
  (cd $dir && env "$@" PYTHONPATH=$PWD timeout -k 10 150 python bench.py --steps 300 --warmup 30 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])") 2>&1 | tee -a gpurun_out/ab3.txt
}
rm -f gpurun_out/ab3.txt
for r in 1 2; do
run "a300e0a" _bisect/a300 MDA_X=1
run "HEAD" . MDA_X=1
run "HEAD perm8 off" . MDA_HALO_PERM8=0
run "HEAD deep off" . MDA_GLDS_DEEP=0
run "HEAD pack extras off" . MDA_PACK_EXTRAS=0
run "HEAD head ksplit 1" . MDA_HEAD_KSPLIT=1
done
exit 0
