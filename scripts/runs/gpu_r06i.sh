#!/bin/bash
# round 6 (i): the driver's SCALE invocation rehearsed on one GPU -- plain `bench.py --gpus 8` (the
# launcher starts 8 ranks) with 8 REAL RCCL ranks sharing the GPU over RCCL's socket transport
# (GOLHIP_RCCL_SHARED_GPU=1), weak-scaling board 4096 x 4096*8 (oracle golden registered), then
# --gpus 4 the same way
set -u
O=gpurun_out/r06i
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for N in 8 4; do
  GOLHIP_RCCL_SHARED_GPU=1 $G 400 $O/bench_plain_${N}.log python -u bench.py --gpus $N --size 4096 --steps 20 --warmup 5 \
    --no-strong --preheat-ms 20 --comm-timeout-ms 120000 --launch-deadline-s 360 || exit $?
  grep '^{' $O/bench_plain_${N}.log > $O/bench_plain_${N}.json || true
  python3 -c "import json;d=json.load(open('$O/bench_plain_${N}.json'));print(d['n_gpus'],d['value'],d['transport'],d['parity'],[r['timed_ms'] for r in d['per_rank']])" || true
done
