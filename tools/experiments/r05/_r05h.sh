set -e
O=gpurun_out/r05h; mkdir -p $O
export TMPDIR=/tmp
F5=filterFrame_2d_float_5x5_quarterCtu
C="2:full:pinned:$F5:2 2:full:pinned 1:full:pinned 2:dec:pinned:$F5:2"
for v in default noext; do
  case $v in default) E="";; noext) E="MIPGPU_EXT_DONE=0";; esac
  env $E timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 $C | sed "s/^/$v /" | cut -c1-330 | tee -a $O/rates.txt
done
COMMON="--no-cpu-baseline --no-reference-gpu --no-latency --no-filter --steps 10 --warmup 2 --allow-knobs"
for v in default noext; do
  case $v in default) E="";; noext) E="MIPGPU_EXT_DONE=0";; esac
  env $E timeout -k 10 300 python bench.py $COMMON --frames-per-step 2 --refs-filter $F5 --kernel-idx 2 > $O/bench_$v.json 2>$O/bench_$v.err
  python3 -c "import json; d=json.load(open('$O/bench_$v.json')); print('$v', d['value'], d['end_to_end'])" | cut -c1-300
done
rm -rf /tmp/tr
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr -o t --output-format csv -- python -u tools/e2e_probe.py --reps 1 2:full:pinned:$F5:2 > /dev/null 2>$O/tr.err
python3 tools/trace_timeline.py /tmp/tr --last 40 > $O/timeline.txt
echo done
