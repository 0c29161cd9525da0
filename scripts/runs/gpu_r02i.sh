#!/bin/bash
# Small-board latency study (configs[1] 5120^2, configs[4] 4096^2 with per-turn counts) + the
# production K=16 PMC passes (VALU issued, effective clock, HBM traffic).
set -u
O=gpurun_out/r02i
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 300 $O/smoke.log python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
$G 300 $O/tune5120.log python3 scripts/tune_small.py 5120 2,4,6,8,12,16 0,8,16,32 2048 || exit $?
$G 300 $O/tune4096.log python3 scripts/tune_small.py 4096 4,8,12,16 0,8,16 2048 || exit $?
GOLHIP_SPLIT=1 $G 300 $O/tune5120_nosplit.log python3 scripts/tune_small.py 5120 16 0,16,32 2048 || exit $?
for K in 16 8 4; do
  $G 200 $O/tl$K.log rocprofv3 --kernel-trace --output-format csv -d $O/tl$K -o tl -- python3 scripts/profile_small.py 5120 $K 4096 counts || exit $?
  python3 scripts/launch_timeline.py $O/tl$K 200 > $O/timeline_k$K.txt 2>&1
done
$G 600 $O/pmc16.log scripts/pmc_passes.sh 16 || exit $?
python3 scripts/pmc_summary.py gpurun_out/pmc_k16 16 536870912 $O/pmc_k16.json 65536x65536_k16 > $O/pmc16_summary.log 2>&1
echo done
