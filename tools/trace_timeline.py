#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --memory-copy-trace run (CSV output) as per-segment
timelines: the trace is cut into segments at idle gaps (tools/e2e_probe.py sleeps 0.2 s
between cases); for each segment it prints the busy time per operation type, the span, and
the last N operations (start and duration in microseconds from the first of them, type,
stream), so the overlap of uploads, searches and downloads can be read directly.

    python tools/trace_timeline.py TRACE_DIR [--last 40] [--gap-ms 50]"""
import argparse
import csv
import glob
import os
from collections import defaultdict


def short(name):
    n = name.split("(")[0]
    for key in ("mip_search_kernel", "dec_split_kernel", "best_mode_kernel", "filter_kernel", "fixup_kernel"):
        if key in name:
            return key.replace("_kernel", "")
    return n[-32:]


def load(d):
    ev = []
    for path in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                       r.get("Stream_Id") or r.get("Queue_Id", "?")))
    for path in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        rd = csv.DictReader(open(path))
        for r in rd:
            dirn = r.get("Direction", "")
            kind = "H2D" if "HOST_TO_DEVICE" in dirn else ("D2H" if "DEVICE_TO_HOST" in dirn else dirn[-12:] or "copy")
            nbytes = r.get("Bytes") or r.get("Size") or r.get("Copy_Bytes") or ""
            if nbytes:
                kind += "(%.1fMB)" % (int(nbytes) / 1e6)
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, r.get("Stream_Id", "?")))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--last", type=int, default=40)
    ap.add_argument("--gap-ms", type=float, default=50.0)
    a = ap.parse_args()
    ev = load(a.trace_dir)
    segs, cur, end = [], [], None
    for e in ev:
        if cur and e[0] - end > a.gap_ms * 1e6:
            segs.append(cur)
            cur = []
        cur.append(e)
        end = e[1] if end is None or not cur[:-1] else max(end, e[1])
    if cur:
        segs.append(cur)
    for i, s in enumerate(segs):
        busy = defaultdict(float)
        cnt = defaultdict(int)
        for st, en, k, _ in s:
            base = k.split("(")[0]
            busy[base] += (en - st) / 1e3
            cnt[base] += 1
        span = (max(e[1] for e in s) - s[0][0]) / 1e3
        print("== segment %d: %d ops, span %.1f us; busy us (count): %s" % (
            i, len(s), span, ", ".join("%s %.1f (%d)" % (k, busy[k], cnt[k]) for k in sorted(busy))))
        tail = s[-a.last:]
        t0 = tail[0][0]
        for st, en, k, strm in tail:
            print("  %9.1f %8.1f  %-22s stream %s" % ((st - t0) / 1e3, (en - st) / 1e3, k, strm))


if __name__ == "__main__":
    main()
