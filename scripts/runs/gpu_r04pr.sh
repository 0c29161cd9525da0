#!/bin/bash
# round 4 (pr): configs[0] call timeline (kernel + memory-copy trace)
set -u
O=gpurun_out/r04pr
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 120 $O/plain.log python3 -u scripts/trace_cfg0.py || exit $?
cat $O/plain.log
$G 200 $O/trace.log rocprofv3 --kernel-trace --memory-copy-trace -d $O/prof -o run -- python3 -u scripts/trace_cfg0.py || exit $?
grep "us per call" $O/trace.log
