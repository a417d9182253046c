# the whole -m gpu suite as the driver runs it, plus smoke()
set -u
mkdir -p gpurun_out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_all.log 2>&1; rc=$?
tail -3 gpurun_out/pt_all.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAILED" gpurun_out/pt_all.log | head -60; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -2 gpurun_out/smoke.log; exit $rc
