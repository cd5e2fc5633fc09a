#!/bin/bash
# Round 6: per-class PMC census (tools/shape_pmc.sh) of the four-wave (MIP_SIX_WAVES 0) and the
# six-wave (default) builds, profiling variants.
set -uo pipefail
cd "$(dirname "$0")/../../.."
for v in s0 s3; do
  echo "## $v"
  MIPGPU_LIB=$PWD/tools/bin/lib_prof_$v.so OUT=gpurun_out/${OUTTAG:-r06shape}/$v timeout -k 10 900 bash tools/shape_pmc.sh > gpurun_out/${OUTTAG:-r06shape}_$v.txt 2>&1 || { tail -20 gpurun_out/${OUTTAG:-r06shape}_$v.txt; exit 1; }
  cat gpurun_out/${OUTTAG:-r06shape}_$v.txt | tail -20
done
