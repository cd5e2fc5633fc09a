set -e
for t in none init alloc stream d2h d2h_pinned; do
  a=""; [ $t != none ] && a="--torch $t"
  timeout -k 10 200 python -u tools/e2e_probe.py --reps 3 $a 1:full:pinned 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['fps'], d['fps_all'])"
done
