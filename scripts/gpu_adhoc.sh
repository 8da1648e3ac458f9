export PYTHONPATH=$PWD TMPDIR=/tmp
for r in 1 2 3; do for w in 3 2 1; do
  echo -n "eager $w: "
  MDA_WARMUP_EAGER=$w timeout -k 10 120 python bench.py --steps 20 --warmup 5 2>/dev/null | grep '^{' | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d.get('final_loss'))"
done; done
