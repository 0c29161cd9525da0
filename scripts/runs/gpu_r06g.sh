#!/bin/bash
# round 6 (g): where the per-turn counts cost goes on a narrow board's long call (512^2, 4096 turns
# with and without counts): kernel trace + stats of each
set -u
O=gpurun_out/r06g
mkdir -p $O
export TMPDIR=/tmp
G=scripts/guard.sh
for C in counts nocounts; do
  $G 120 $O/trace_512_$C.log rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/r06g_$C -o t -- python3 scripts/profile_small.py 512 16 4096 $C || exit $?
  find /tmp/r06g_$C -name "t_kernel_stats.csv" -exec cp {} $O/kernel_stats_512_$C.csv \;
  find /tmp/r06g_$C -name "t_memory_copy_stats.csv" -exec cp {} $O/copy_stats_512_$C.csv \;
  find /tmp/r06g_$C -name "t_kernel_trace.csv" -exec cp {} $O/kernel_trace_512_$C.csv \;
done
ls -la $O
