#!/bin/bash
# 8 x MI355X (one node, xGMI): one process per GPU via torchrun, RCCL all-reduce; global batch 96.
mkdir -p checkpoints
python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \
  train.py --name raft-chairs --stage chairs --validation chairs --num_steps 100000 --batch_size 96 \
  --lr 0.0004 --image_size 368 496 --wdecay 0.0001 --mixed_precision --hipgraph
