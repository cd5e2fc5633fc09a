set -e
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "pipeline or async or per_frame or ticket or pageable or decisions or contract or dropped" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
F5=filterFrame_2d_float_5x5_quarterCtu
C="1:dec:pinned 1:full:pinned 2:dec:pinned:$F5:2 1:dec:pageable"
for v in default inline nofence device; do
  case $v in default) E="";; inline) E="MIPGPU_DEC_INLINE=1";; nofence) E="MIPGPU_SLOT_EVENTS=nofence";; device) E="MIPGPU_SLOT_EVENTS=device";; esac
  echo "== $v"; env $E timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 $C | sed "s/^/$v /" | tee -a $O/rates.txt
done
export TMPDIR=/tmp
for v in default nofence; do
  case $v in default) E="";; nofence) E="MIPGPU_SLOT_EVENTS=nofence";; esac
  rm -rf /tmp/tr_$v
  env $E timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr_$v -o t --output-format csv -- python -u tools/e2e_probe.py --reps 1 1:dec:pinned > /dev/null 2>$O/tr_$v.err
  python3 tools/trace_timeline.py /tmp/tr_$v --last 40 > $O/timeline_$v.txt
done
echo done
