#!/bin/bash
# round 4 (j): why predict_scaling's ring of one runs 1000 turns in ~41 ms when a process holding
# only the ring engine runs them in 35.6 (r04i): kernel trace of predict (queue ids per stream),
# then predict with more hardware queues per process
set -u
O=gpurun_out/r04j
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 200 $O/predict_trace.log rocprofv3 --kernel-trace --output-format csv -d /tmp/r04j_t -o t -- python3 scripts/predict_scaling.py 1 1000 0 || exit $?
grep "^{\"shape" $O/predict_trace.log | cut -c1-250
python3 scripts/ring_timeline.py /tmp/r04j_t 4 150 > $O/timeline_predict.txt 2>&1
cut -c1-700 $O/timeline_predict.txt
GPU_MAX_HW_QUEUES=8 $G 300 $O/predict_hwq8.log python3 scripts/predict_scaling.py 5 20,1000 160 1,8 || exit $?
grep "^{\"shape" $O/predict_hwq8.log | cut -c1-250
