#!/bin/bash
# Multi-process rehearsal of bench.py on a one-GPU box: 2 ranks on the same GPU.  RCCL
# refuses two ranks on one device ("Duplicate GPU detected"), so the rehearsal runs the
# same torch.distributed path over gloo; the 8-GPU driver run uses nccl (RCCL).
mkdir -p gpurun_out/mr
export HSA_ENABLE_IPC_MODE_LEGACY=0
GPMDM_BENCH_BACKEND=gloo timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 \
  > gpurun_out/mr/gloo.json 2> gpurun_out/mr/gloo.err
rc=$?; echo "gloo rc=$rc"
grep -i "error\|Traceback" gpurun_out/mr/gloo.err | head -5
cat gpurun_out/mr/gloo.json
exit $rc
