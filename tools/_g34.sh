# full GPU suite at HEAD (dense cross terms on by default where they pay)
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt34.log 2>&1; rc=$?
tail -3 gpurun_out/pt34.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\|FAILED" gpurun_out/pt34.log | head -80; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke34.log 2>&1; rc=$?
tail -2 gpurun_out/smoke34.log; exit $rc
