set -e
O=gpurun_out/r05v; mkdir -p $O
F5=filterFrame_2d_float_5x5_quarterCtu
C="8:full:pageable 8:full:pinned 1:dec:pageable 2:full:pageable:$F5:2 32:full:pageable"
for lib in vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_pieces.so vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_pieces.so; do
  MIPGPU_LIB=$PWD/$lib timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --torch init $C 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$(basename $lib)', d['case'][:24], d['fps'], d['fps_all'], d['enqueue_ms'][-1], d['wait_ms'][-1])" | tee -a $O/ab.txt
done
export TMPDIR=/tmp
rm -rf /tmp/pt
MIPGPU_STAGE_STATS=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/pt -o pipe --output-format csv -- python -u tools/e2e_probe.py --reps 1 --torch init 8:full:pageable 8:full:pinned > $O/trace_rates.jsonl 2> $O/trace.err || { tail $O/trace.err; exit 1; }
python3 tools/trace_timeline.py /tmp/pt --last 150 > $O/timeline.txt
echo done
