#!/bin/bash
# Round 6 final GPU pass: tests + smoke + kernel trace / PMC + bench line + small launches
# (tools/final_round.sh), the config sweep, the multi-rank rehearsal (end-to-end legs at N > 1),
# queued one-frame calls merged / not.  Two gpurun calls: final.sh a, then final.sh b.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06final; mkdir -p $O
if [ "${1:-a}" = a ]; then OUT=$O bash tools/final_round.sh; exit $?; fi
echo "== config sweep $(date +%T)"
OUT=$O bash tools/config_sweep.sh > $O/configs.log 2>&1 || { tail -20 $O/configs.log; exit 1; }
tail -3 $O/configs.log | cut -c1-300
echo "== multirank $(date +%T)"
OUT=$O bash tools/multirank_rehearsal.sh > $O/multirank.log 2>&1 || { tail -20 $O/multirank.log; exit 1; }
grep -E "^==|aggregate" $O/multirank.log | cut -c1-300
echo "== merge rates $(date +%T)"
OUTTAG=r06final/merge DDS=1 bash tools/experiments/r06/k.sh > $O/merge.log 2>&1 || { tail -20 $O/merge.log; exit 1; }
tail -12 $O/merge.log
echo "== four-wave vs default $(date +%T)"
OUTTAG=r06final/ab_s0 S6LIB=vvc-mip-gpu_amd/lib/libmipgpu.so EXTRA_LIBS=tools/bin/lib_s0.so bash tools/experiments/r06/s6.sh > $O/ab_s0.log 2>&1 || { tail -20 $O/ab_s0.log; exit 1; }
tail -9 $O/ab_s0.log
echo "== done $(date +%T)"
