set -e
O=gpurun_out/r05j; mkdir -p $O
export TMPDIR=/tmp
F5=filterFrame_2d_float_5x5_quarterCtu
for t in "" "--torch"; do
  timeout -k 10 200 python -u tools/e2e_probe.py --reps 3 $t 2:full:pinned:$F5:2 1:full:pinned | cut -c1-200 | sed "s/^/torch=$t /"
done
for t in notorch torch; do
  rm -rf /tmp/tr_$t; a=""; [ $t = torch ] && a="--torch"
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr_$t -o t --output-format csv -- python -u tools/e2e_probe.py --reps 1 $a 2:full:pinned:$F5:2 > /dev/null 2>$O/tr_$t.err
  python3 tools/trace_timeline.py /tmp/tr_$t --last 12 > $O/timeline_$t.txt
  grep "== segment" $O/timeline_$t.txt | tail -3 | cut -c1-250
done
echo done
