#!/bin/bash
# round 2 (aj): per-wave LDS count slots (no contended LDS atomics): slab tests, then A/B vs lib_prev
set -o pipefail
O=gpurun_out/r02aj; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "slab or small_board or register or count" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || exit 1
for rep in 1 2; do
  for L in lib_prev lib; do
    GOLHIP_LIB=distributed-gol_amd/$L/libgolhip.so timeout -k 10 120 python3 scripts/cfg2_time.py > $O/$L.$rep.json 2> $O/$L.$rep.err || { echo "FAIL $L"; tail -3 $O/$L.$rep.err; exit 1; }
    GOLHIP_LIB=distributed-gol_amd/$L/libgolhip.so timeout -k 10 120 python3 scripts/cfg2_time.py cfg5 > $O/c5_$L.$rep.json 2> $O/c5_$L.$rep.err || { echo "FAIL c5 $L"; tail -3 $O/c5_$L.$rep.err; exit 1; }
    echo "$L $rep $(cat $O/$L.$rep.json) $(cat $O/c5_$L.$rep.json)"
  done
done
