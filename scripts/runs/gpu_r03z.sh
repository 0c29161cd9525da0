#!/bin/bash
# round 3 (z): is the hot kernel bound by bit activity?  (1) a chip-wide v_bitop3 stream on random
# vs zero operands (cycles per VALU at the in-kernel shader clock); (2) the production stencil on an
# empty, a sparse and a random board (same instruction stream)
set -u
O=gpurun_out/r03z
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
$G 120 $O/ubench_toggle.log scripts/ubench_toggle 5 || exit $?
grep "^{" $O/ubench_toggle.log
$G 300 $O/density_k12.log python3 scripts/density_ab.py 65536 12 7 || exit $?
tail -3 $O/density_k12.log
