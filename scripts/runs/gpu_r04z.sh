#!/bin/bash
# round 4 (z): the split step's join of the boundary bands as an event wait (production) vs a
# stream write/wait of a device word (tuning GOLHIP_JOIN=1): ring parity under the knob, the ring's
# timeline and the prediction with each
set -u
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
TL=distributed-gol_amd/lib_tuning/libgolhip.so
GOLHIP_LIB=$TL GOLHIP_JOIN=1 $G 300 $O/ring_join1.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "ring_of_one" --timeout 250 --timeout-method thread || exit $?
tail -2 $O/ring_join1.log
grep -q " passed" $O/ring_join1.log && ! grep -qE " failed| error" $O/ring_join1.log || exit 1
for j in 0 1; do
  GOLHIP_LIB=$TL GOLHIP_JOIN=$j $G 200 $O/run_j$j.log rocprofv3 --kernel-trace --output-format csv -d /tmp/r04z_$j -o t -- python3 scripts/ring_timeline.py run 65536 1000 1 8 || exit $?
  python3 scripts/ring_timeline.py /tmp/r04z_$j 2 70 > $O/timeline_j$j.txt 2>&1
  echo "join=$j"; tail -1 $O/timeline_j$j.txt | cut -c1-400
  GOLHIP_LIB=$TL GOLHIP_JOIN=$j GPU_MAX_HW_QUEUES=8 $G 300 $O/predict_j$j.log python3 scripts/predict_scaling.py 5 20,1000 0 || exit $?
  grep "^{\"shape" $O/predict_j$j.log | cut -c1-250
done
