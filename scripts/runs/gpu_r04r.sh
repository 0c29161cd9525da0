#!/bin/bash
# round 4 (r): interior enqueued before the RCCL exchange: ring parity + fail-fast, the raw tail
# timeline, the rank rehearsal at 20/5 and 1000, the prediction
set -u
O=gpurun_out/r04r
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/ring_tests.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_failfast.py -m gpu -v -k "ring or stall or never_joins" --timeout 250 --timeout-method thread || exit $?
grep -E "passed|failed" $O/ring_tests.log | tail -2
grep -q " passed" $O/ring_tests.log && ! grep -qE " failed| error" $O/ring_tests.log || exit 1
$G 200 $O/run20.log rocprofv3 --kernel-trace --output-format csv -d /tmp/r04r_t -o t -- python3 scripts/ring_timeline.py run 65536 20 1 5 || exit $?
python3 scripts/ring_timeline.py /tmp/r04r_t tail 8 > $O/tail20_ring.txt 2>&1; cat $O/tail20_ring.txt
F="--no-cpu --no-sweep --no-strong --no-configs --no-flips"
for st in "20 5" "1000 8"; do set -- $st
  $G 200 $O/plain_s$1.log python3 bench.py --steps $1 --warmup $2 $F || exit $?
  GOLHIP_RING_SELF=1 $G 200 $O/rehearsal_s$1.log python3 bench.py --steps $1 --warmup $2 --pg-always $F || exit $?
done
for f in plain_s20 rehearsal_s20 plain_s1000 rehearsal_s1000; do grep '^{' $O/$f.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); i=d["instrumented_pass"]; print("'$f'", d["value"], d["ms_per_step"], i["kernel_ms"], d["parity"]["ok"], d["parity"].get("digest_ok"))'; done
GPU_MAX_HW_QUEUES=8 $G 300 $O/predict.log python3 scripts/predict_scaling.py 5 20,1000 160 || exit $?
grep "^{\"shape" $O/predict.log | cut -c1-250
