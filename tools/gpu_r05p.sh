#!/bin/bash
# round 5: the rs.h host-path tests (incl. edited matrices over many chunks) and the driver's own
# torch.distributed.run launch of bench.py at N=1 (RCCL process group on the one GPU)
set -o pipefail
OUT=gpurun_out/${1:-r05p}; mkdir -p $OUT
source tools/gpu_step.sh
step tests 300 python -u -m pytest tests/test_gpu_rs_host.py -x -q --timeout 120 --timeout-method thread
step torchrun1 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu
tail -c 400 $OUT/torchrun1.log
