set -e
cd /root/repo
OUT=gpurun_out/sp1 bash tools/shape_pmc.sh
MIPGPU_NO_PAIRS=1 OUT=gpurun_out/sp0 bash tools/shape_pmc.sh
