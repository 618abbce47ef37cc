#!/bin/bash
# N > 1 rehearsal on one GPU: 2 ranks of bench.py under torch.distributed.run, gloo carrying the GPU
# gradients (RCCL refuses two ranks on one device) -- exercises GradAllReducer's bucketed launches
# from inside the HIP backward on the side stream, the buffer broadcast, the barriers and the
# max-over-ranks timing with the real models
OUT=gpurun_out/r2s7; mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --model envnet --steps 4 --warmup 2 --no-cpu-baseline \
  --dist-backend gloo > $OUT/envnet.json 2> $OUT/envnet.err || { tail -30 $OUT/envnet.err; exit 1; }
head -c 600 $OUT/envnet.json; echo
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29532 bench.py --gpus 2 --model ast --ast-batch 32 --steps 3 --warmup 2 --no-cpu-baseline \
  --dist-backend gloo > $OUT/ast.json 2> $OUT/ast.err || { tail -30 $OUT/ast.err; exit 1; }
head -c 600 $OUT/ast.json; echo
