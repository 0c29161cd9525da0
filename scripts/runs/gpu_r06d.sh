#!/bin/bash
# round 6 (d): lib_tuning pushed for this call (.gpurunignore line removed): the tuning suite
# against the round-6 tuning library; then the default bench under rocprofv3 --kernel-trace --stats
# (the line's HIP-event launch average vs rocprof's), and the driver's command again (cfg5_host with
# the 2 s tick inside the pause)
set -u
O=gpurun_out/r06d
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 700 $O/tuning.log python -u -m pytest tests/test_gpu_tuning.py tests/test_gpu_failfast.py -m gpu -x -q --timeout 280 --timeout-method thread || exit $?
tail -3 $O/tuning.log
$G 400 $O/bench_prof.log rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/r06d_prof -o b -- python3 bench.py --no-cpu --no-configs --no-host --no-flips || exit $?
grep '^{' $O/bench_prof.log > $O/bench_under_rocprof.json || true
find /tmp/r06d_prof -name "b_kernel_stats.csv" -exec cp {} $O/bench_kernel_stats.csv \;
$G 400 $O/bench20.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
grep '^{' $O/bench20.log > $O/bench20.json || true
python3 -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'],d['roofline']['frac'],json.dumps(d['cfg5_host']['reference'])[:1200])" || true
