#!/bin/bash
# New round-3 GPU tests first (config 1, full-size learner, tightened v7/sp7 agreement), then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_episode.py tests/test_gpu_learner.py tests/test_gpu_rollout.py::test_rollout_v7_split_bf16_gru_matches_fp32 tests/test_gpu_selfplay.py::test_selfplay_sp7_split_bf16_matches_fp32 -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/new_tests.log 2>&1 || { tail -40 gpurun_out/new_tests.log; exit 1; }
tail -2 gpurun_out/new_tests.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
