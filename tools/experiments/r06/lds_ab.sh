#!/bin/bash
# Round 6: per-class LDS bank conflicts (tools/shape_lds.sh) of the six-wave default and the
# four-wave build (profiling variants), one box.
set -uo pipefail
cd "$(dirname "$0")/../../.."
for v in libmipgpu_prof lib_prof_s0; do
  echo "## $v"
  MIPGPU_LIB=$PWD/tools/bin/$v.so OUT=gpurun_out/${OUTTAG:-r06lds}/$v timeout -k 10 600 bash tools/shape_lds.sh > gpurun_out/${OUTTAG:-r06lds}_$v.txt 2>&1 || { tail -20 gpurun_out/${OUTTAG:-r06lds}_$v.txt; exit 1; }
  tail -19 gpurun_out/${OUTTAG:-r06lds}_$v.txt
done
