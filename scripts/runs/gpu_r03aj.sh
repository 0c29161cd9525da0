#!/bin/bash
# round 3 (aj): PMC passes of the production K = 14 launch (the new bulk depth at 65536^2)
set -u
O=gpurun_out/r03aj
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/pmc14.log bash scripts/pmc_passes.sh 14 || exit $?
echo done
