#!/bin/bash
# Round 6: standalone reproducer of the half-speed transfers after a large device free.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06n; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 tools/bin/free_repro 20 > $O/repro.jsonl 2> $O/repro.err || { cat $O/repro.err; exit 1; }
cat $O/repro.jsonl
rm -rf /tmp/trn
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/trn -o t --output-format csv -- tools/bin/free_repro 20 > $O/repro_traced.jsonl 2> $O/repro_traced.err || { tail $O/repro_traced.err; exit 1; }
python - <<'P'
import csv, glob, collections
rows = []
for p in glob.glob("/tmp/trn/**/*memory_copy_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
for p in glob.glob("/tmp/trn/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        rows.append(dict(r, Direction="KERNEL " + r["Kernel_Name"][:40]))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
print("columns:", sorted(rows[0].keys())[:30] if rows else None)
# group consecutive copies of the same direction and size: count, mean GB/s, engine fields
groups = []
for r in rows:
    key = (r.get("Direction"), r.get("Size") or r.get("Bytes"), r.get("Src_Agent_Id") or r.get("Source_Agent_Id"), r.get("Dst_Agent_Id") or r.get("Destination_Agent_Id"))
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    if groups and groups[-1][0] == key:
        groups[-1][1].append(dur)
    else:
        groups.append([key, [dur]])
for key, durs in groups:
    n = int(key[1]) if key[1] and key[1].isdigit() else 0
    print(key, len(durs), "mean %.1f us" % (1e6 * sum(durs) / len(durs)), ("%.1f GB/s" % (n / (sum(durs) / len(durs)) / 1e9)) if n else "")
P
