set -e
O=gpurun_out/r05aq; mkdir -p $O
run() { timeout -k 10 300 python -u tools/e2e_probe.py --reps 3 "$@" 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$*'[:60], '|', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt; }
run 1:full:pinned 128:dec:pinned:mb=384 1:full:pinned
run 1:full:pinned 4:dec:pinned 1:full:pinned
run 1:full:pinned 128:full:pinned:mb=384 1:full:pinned
MIPGPU_NO_TORCH=1 run 1:full:pinned 128:dec:pinned:mb=384 1:full:pinned
echo done
