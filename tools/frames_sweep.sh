for B in 32 64 128 256; do
  timeout -k 10 120 python bench.py --frames-per-step $B --steps 10 --warmup 2 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B', d['value'], d['roofline']['kernel_ms_per_launch'])"
done
