set -e
O=gpurun_out/r05r; mkdir -p $O
MIPGPU_LIB=$PWD/tools/bin/lib_six2.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "small_configs or full_size or edge or small_launch" > $O/pytest_six2.log 2>&1 || { tail -40 $O/pytest_six2.log; exit 1; }
tail -1 $O/pytest_six2.log
FRAMES=384 timeout -k 10 600 tools/ab_bench.sh 3 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_tabg.so tools/bin/lib_six2.so tools/bin/lib_six.so 2>&1 | tee $O/ab_384.txt
echo done
