#!/bin/bash
# Round-3 league check on one GPU: GPU tests, the default bench (config 2 + league leg + CPU baselines), the bench
# under torch.distributed.run with one rank (the league's collectives over RCCL at world size 1), and a world-2
# gloo rehearsal with both ranks on cuda:0. Each GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/tests.log 2>&1 || { tail -30 gpurun_out/tests.log; exit 1; }
tail -2 gpurun_out/tests.log
timeout -k 10 400 python bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/bench_n1.json 2> gpurun_out/bench_n1.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench_n1.err; exit 1; }
cat gpurun_out/bench_n1.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29511 bench.py --gpus 1 --steps 10 --warmup 2 --no-cpu-baseline \
    > gpurun_out/bench_rccl1.json 2> gpurun_out/bench_rccl1.err || { echo "rccl world-1 bench failed"; tail -20 gpurun_out/bench_rccl1.err; exit 1; }
cat gpurun_out/bench_rccl1.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo --device 0 --no-cpu-baseline \
    > gpurun_out/rehearsal_2.json 2> gpurun_out/rehearsal_2.err || { echo "rehearsal 2 failed"; tail -20 gpurun_out/rehearsal_2.err; exit 1; }
cat gpurun_out/rehearsal_2.json
