set -e
O=gpurun_out/r05q; mkdir -p $O
MIPGPU_LIB=$PWD/tools/bin/lib_six.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_six.log 2>&1 || { tail -40 $O/pytest_six.log; exit 1; }
tail -1 $O/pytest_six.log
FRAMES=384 timeout -k 10 400 tools/ab_bench.sh 3 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_six.so 2>&1 | tee $O/ab_384.txt
FRAMES=128 EXTRA="--refs-filter filterFrame_2d_float_5x5_quarterCtu --kernel-idx 2" timeout -k 10 400 tools/ab_bench.sh 2 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_six.so 2>&1 | tee $O/ab_alt128.txt
FRAMES=32 timeout -k 10 400 tools/ab_bench.sh 2 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_six.so 2>&1 | tee $O/ab_32.txt
FRAMES=2 timeout -k 10 400 tools/ab_bench.sh 2 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_six.so 2>&1 | tee $O/ab_2.txt
echo done
