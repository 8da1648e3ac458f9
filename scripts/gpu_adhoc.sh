export TMPDIR=/tmp
for w in _bisect/r4 _bisect/e79; do
  echo "== $w"
  (cd $w && PYTHONPATH=$PWD ARM=default TRIALS=4 timeout -k 10 300 python -u scripts/debug/ofd_nan.py > ../../gpurun_out/ofd_nan_$(basename $w).log 2>&1) || exit 1
  grep -v "amdgpu.ids\|WARN" gpurun_out/ofd_nan_$(basename $w).log | tail -6
done
