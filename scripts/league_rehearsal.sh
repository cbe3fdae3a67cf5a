#!/bin/bash
# Multi-rank league rehearsal on ONE GPU: N ranks (gloo collectives, every rank on cuda:0) run bench.py's
# league mode end to end -- the code path the driver's 2/4/8-GPU runs take with RCCL, minus the transport.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for n in ${RANKS:-2 4}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 \
    --master-port $((29500 + n)) bench.py --gpus $n --steps ${STEPS:-10} --warmup 2 --backend gloo --device 0 \
    --no-cpu-baseline > gpurun_out/rehearsal_$n.json 2> gpurun_out/rehearsal_$n.err || { echo "rehearsal $n failed"; tail -20 gpurun_out/rehearsal_$n.err; exit 1; }
  cat gpurun_out/rehearsal_$n.json
done
