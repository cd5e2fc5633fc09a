#!/bin/bash
# Build an A/B variant of libmipgpu.so with extra compiler flags for every engine source:
#   tools/build_variant.sh OUT.so [extra hipcc flags...]
# e.g. the profiling build that honours MIPGPU_SHAPE_FILTER / MIPGPU_NO_PAIRS (wrong tables
# by design; the release library refuses them):
#   tools/build_variant.sh tools/bin/libmipgpu_prof.so -DMIPGPU_PROFILING_KNOBS
# The variant's build ID names the extra flags (knobs:...), so bench.py and profiles/ never
# take it for the release library.
set -euo pipefail
cd "$(dirname "$0")/../vvc-mip-gpu_amd"
out=$1; shift
case "$out" in /*) ;; *) out="$OLDPWD/$out" ;; esac
mkdir -p "$(dirname "$out")"
tmp=$(mktemp -d)
trap 'rm -rf "$tmp"' EXIT
id="$(make -s KNOBS="$*" build-id)"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc $*"
pids=()
for s in mip_search mip_filter mip_fixup; do
  /opt/rocm/bin/hipcc $F -c -o "$tmp/$s.o" "csrc/$s.hip" & pids+=($!)
done
/opt/rocm/bin/hipcc $F -DMIP_SIX_WAVES=0 -DMIP_FOUR_WAVE_TWIN=1 -c -o "$tmp/mip_search_four.o" csrc/mip_search.hip \
  2> >(grep -v "macro redefined\|^ *[0-9]* | \|^ *| \|note: previous definition\|warning generated\|^<command line>" >&2) & pids+=($!)
/opt/rocm/bin/hipcc $F "-DMIPGPU_BUILD_ID=\"$id\"" -c -o "$tmp/mipgpu.o" csrc/mipgpu.cpp & pids+=($!)
for p in "${pids[@]}"; do wait "$p" || { echo "build_variant: a compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out" "$tmp"/*.o
echo "built $out ($id)"
