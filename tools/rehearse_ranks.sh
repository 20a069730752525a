#!/bin/bash
# The N > 1 bench path (bench.py under torch.distributed.run, one rank per "GPU") rehearsed on ONE GPU:
# every rank drives cuda:0 and the all-to-all is staged through host memory over gloo
# (NTT_BENCH_EXCHANGE=host; RCCL refuses two ranks on one device).  Checks that the launch, the rank
# plans, the barrier / max-over-ranks timing and the JSON line work for N = 2, 4, 8; the times are
# NOT the product's (host-staged exchange, N ranks sharing one GPU).
set -o pipefail
O=${O:-gpurun_out/rehearse}
mkdir -p $O
for N in 2 4 8; do
  NTT_BENCH_EXCHANGE=host timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N \
    --master-addr 127.0.0.1 --master-port $((29600 + N)) bench.py --gpus $N --steps 10 --warmup 5 \
    > $O/bench_n$N.log 2>&1 || { echo "N=$N failed"; tail -20 $O/bench_n$N.log; exit 1; }
  grep '^{' $O/bench_n$N.log | tail -1
done
