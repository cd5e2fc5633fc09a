#!/bin/bash
# Round 6: the half-speed transfer state -- which streams / which pinned-allocation history.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06o; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 tools/bin/free_repro remedy >> $O/remedy.jsonl 2>> $O/remedy.err || { cat $O/remedy.err; exit 1; }
  echo "--" >> $O/remedy.jsonl
done
for i in 1 2; do timeout -k 10 120 tools/bin/free_repro 20 >> $O/repro.jsonl 2>> $O/repro.err || exit 1; echo "--" >> $O/repro.jsonl; done
python -c "
import json
for f in ('$O/remedy.jsonl','$O/repro.jsonl'):
    for l in open(f):
        if l.startswith('--'): print('--'); continue
        d=json.loads(l); print('%-52s d2h %5.1f h2d %5.1f' % (d['phase'], d['d2h_GBps'], d['h2d_GBps']))
"
export TMPDIR=/tmp; rm -rf /tmp/tro
timeout -k 10 120 rocprofv3 --memory-copy-trace -d /tmp/tro -o t --output-format csv -- tools/bin/free_repro remedy > /dev/null 2>&1
python -c "
import csv,glob
p=glob.glob('/tmp/tro/**/*memory_copy_trace.csv', recursive=True)[0]
rows=list(csv.DictReader(open(p)))
print(list(rows[0].keys()))
for r in rows[:3]+rows[-3:]: print(r)
"
