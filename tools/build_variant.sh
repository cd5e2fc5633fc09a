#!/bin/bash
# Build an A/B variant of libmipgpu.so with extra compiler flags for the search kernel:
#   tools/build_variant.sh OUT.so [extra hipcc flags...]
set -euo pipefail
cd "$(dirname "$0")/../vvc-mip-gpu_amd"
out=$1; shift
tmp=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -I../include -Icsrc "$@" -c -o $tmp/mip_search.o csrc/mip_search.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$OLDPWD/$out" $tmp/mip_search.o build/mip_filter.o build/mip_fixup.o build/mipgpu.o
rm -rf $tmp
