export PYTHONPATH=$PWD TMPDIR=/tmp
for tf in True False; do
  for r in 1 2; do
    ms=$(timeout -k 10 200 python bench.py --steps 300 --warmup 30 RUNTIME.TEACHER_FIRST $tf 2>/dev/null | grep -o '"ms_per_step": [0-9.]*') || exit 1
    echo "teacher_first=$tf run $r $ms"
  done
done
