#!/bin/bash
# Multi-process rehearsal of bench.py on a one-GPU box: N ranks (default 8) on the same GPU.
# RCCL refuses two ranks on one device ("Duplicate GPU detected"), so the rehearsal runs the
# same torch.distributed path over gloo; the 8-GPU driver run uses nccl (RCCL).
# Usage (on the box): bash tools/rehearse_ranks.sh [N]
n=${1:-8}
mkdir -p gpurun_out/mr
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPMDM_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus $n --steps 5 --warmup 2 --no-cpu-baseline \
  > gpurun_out/mr/gloo$n.json 2> gpurun_out/mr/gloo$n.err
rc=$?; echo "gloo ranks=$n rc=$rc"
grep -i "error\|Traceback" gpurun_out/mr/gloo$n.err | head -5
cat gpurun_out/mr/gloo$n.json
exit $rc
