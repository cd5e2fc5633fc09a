set -e
O=${O:-gpurun_out/r05s}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F5=filterFrame_2d_float_5x5_quarterCtu
MIPGPU_STAGE_STATS=1 timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --torch init 1:dec:pinned 1:dec:pageable 1:full:pinned 1:full:pageable 2:full:pinned:$F5:2 2:full:pageable:$F5:2 8:full:pageable 32:full:pageable 32:full:pinned > $O/probe.jsonl 2> $O/probe.err
cat $O/probe.jsonl | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['case'], d['fps'], d['fps_all'])"
tail -12 $O/probe.err
echo done
