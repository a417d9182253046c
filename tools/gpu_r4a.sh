#!/bin/bash
# round-4 GPU check: the new streamed / sharded / dense tests, then the presets bench
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_stream.py \
  "tests/test_gpu_multirank.py::test_emulated_out_of_core_ranks_match_oracle" \
  "tests/test_gpu_multirank.py::test_reshard_memory_refusal_is_decided_by_every_rank" \
  "tests/test_gpu_dense.py::test_dense_counts_beyond_8_bits" > gpurun_out/r4a_tests.log 2>&1
rc=$?
tail -15 gpurun_out/r4a_tests.log
[ $rc -le 1 ] || exit $rc
bash tools/bench_presets.sh
