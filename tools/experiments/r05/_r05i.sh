set -e
O=gpurun_out/r05i; mkdir -p $O
export TMPDIR=/tmp
F5=filterFrame_2d_float_5x5_quarterCtu
rm -rf /tmp/tr
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr -o t --output-format csv -- python bench.py --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --steps 3 --warmup 1 --frames-per-step 2 --refs-filter $F5 --kernel-idx 2 > $O/bench.json 2>$O/bench.err
cut -c1-200 $O/bench.json
python3 tools/trace_timeline.py /tmp/tr --last 150 --gap-ms 5 > $O/timeline.txt
head -3 $O/timeline.txt
echo done
