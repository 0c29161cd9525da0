#!/bin/bash
# round 2 (v): A/B of the west word by ds_bpermute (lib_x, -DGOLHIP_WEST_BPERM) vs DPP (lib),
# production variant and the two-step ZIP variant (GOLHIP_VARIANT=9), alternating; then PMC k12.
set -o pipefail
O=gpurun_out/r02v; mkdir -p $O
B="python3 bench.py --no-cpu --no-strong --no-flips --no-configs"
run() {  # name env...
  local n=$1; shift
  env "$@" timeout -k 10 200 $B > $O/$n.json 2> $O/$n.err || { echo "FAIL $n"; tail -3 $O/$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n', d['value'], d['cold_start']['value'], d['parity']['ok'], d['roofline']['avg_launch_us'], d['k_sweep_gcups'])"
}
X=GOLHIP_LIB=distributed-gol_amd/lib_x/libgolhip.so
run dpp1 A=1
run bperm1 $X
run dpp2 A=1
run bperm2 $X
run zip_dpp GOLHIP_VARIANT=9
run zip_bperm GOLHIP_VARIANT=9 $X
./scripts/pmc_passes.sh 12 > $O/pmc12.log 2>&1 || { echo "pmc failed"; tail -3 $O/pmc12.log; exit 1; }
echo done
