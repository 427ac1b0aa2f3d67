#!/bin/bash
# round 6: the driver's bench command timed end to end; the N-rank launcher rehearsed on one GPU
# (2 ranks, gloo, default gather interval and every step); the RCCL gather at world size 1
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/${OUT_TAG:-r6n}
mkdir -p $O
t0=$(date +%s)
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.log 2>&1 || exit 1
echo "driver command wall $(( $(date +%s) - t0 )) s" > $O/walls.txt
t0=$(date +%s)
OPK_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 6 --warmup 2 > $O/rehearse2.log 2>&1 || exit 1
OPK_BENCH_REHEARSE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 6 --warmup 2 --gather-interval 1 > $O/rehearse2_every.log 2>&1 || exit 1
echo "rehearsals wall $(( $(date +%s) - t0 )) s" >> $O/walls.txt
timeout -k 10 300 python bench.py --collective-gather --steps 5 --warmup 2 --no-cpu-baseline --no-extra-configs > $O/collective.log 2>&1 || exit 1
