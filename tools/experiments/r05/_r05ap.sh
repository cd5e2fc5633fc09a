set -e
O=gpurun_out/r05ap; mkdir -p $O
for v in X=1 DEBUG_CLR_LIMIT_BLIT_WG=16 DEBUG_CLR_LIMIT_BLIT_WG=64 X=1 DEBUG_CLR_LIMIT_BLIT_WG=16; do
  env $v timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 1:dec:pinned 4:dec:pinned 128:dec:pinned:mb=384 1:full:pinned 128:full:pinned:mb=384 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
