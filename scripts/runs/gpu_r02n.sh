#!/bin/bash
set -u
O=gpurun_out/r02n
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 400 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py -k "register_ or small_board or graph or count_window" -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" $O/pytest.log && ! grep -q "FAILED\|ERROR" $O/pytest.log || { echo "tests failed"; exit 1; }
$G 300 $O/small_configs.log python3 scripts/small_configs.py || exit $?
for C in counts nc; do
  A=""; [ $C = counts ] && A=counts
  $G 200 $O/tl_$C.log rocprofv3 --kernel-trace --output-format csv -d $O/tl_$C -o tl -- python3 scripts/profile_small.py 5120 16 2048 $A || exit $?
  python3 scripts/launch_timeline.py $O/tl_$C 100 > $O/timeline_$C.txt 2>&1
done
echo done
