set -e
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
b() { MIPGPU_LIB=$PWD/abtest/$1.so timeout -k 10 120 python bench.py $2 --steps 20 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$1 $2', d['value'], d['roofline']['kernel_ms_per_launch'])"; }
for r in 1 2; do for lib in novar var; do b $lib ""; done; done
for lib in novar var; do b $lib "--width 3840 --height 2160 --frames-per-step 8"; done
