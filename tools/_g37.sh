# HEAD record of the full-size config parity vs the C oracle (configs 1-5; 3 and 5 take the dense
# cross terms), then the PMC SQ counters of the headline's kernels
set -u
mkdir -p gpurun_out
timeout -k 10 700 python -u tools/config_runs.py --configs 1,2,3,4,5 > gpurun_out/config_runs37.jsonl 2> gpurun_out/config_runs37.err; rc=$?
cat gpurun_out/config_runs37.jsonl | cut -c1-300
[ $rc -eq 0 ] || { tail -20 gpurun_out/config_runs37.err; exit $rc; }
bash tools/_g35.sh
