#!/usr/bin/env python3
"""Summarise a bounce-ring event trace (MIPGPU_STAGE_TRACE=prefix, csrc/host_stage.h): per
part, when the caller took it (T), enqueued it (P), when the completion thread saw its DMA
done (D) and finished it (C), and the caller's waits for room (W); per call, the span from
its first take to its last part finished.  Times in ms from the first event.

    python tools/stage_trace.py TRACE.txt [--parts 60] [--from-call C]"""
import argparse
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--parts", type=int, default=60)
    ap.add_argument("--from-call", type=int, default=0)
    a = ap.parse_args()
    head = ""
    ev = []
    for line in open(a.trace):
        if line.startswith("#"):
            head = line.strip()
            continue
        t, k, seq, off, nb, call, down = line.split()
        ev.append((float(t), k, int(seq), int(off), int(nb), int(call), down == "1"))
    t0 = ev[0][0]
    parts = defaultdict(dict)
    waits = []
    for t, k, seq, off, nb, call, down in ev:
        if k == "W":
            waits.append(((t - t0) * 1e3, seq))
            continue
        p = parts[seq]
        p[k] = (t - t0) * 1e3
        p.update(off=off, nb=nb, call=call, down=down)
    print(head)
    print("%6s %5s %3s %10s %7s %9s %9s %9s %9s" % ("part", "call", "dir", "off MB", "MB", "T", "P", "D", "C"))
    shown = 0
    for seq in sorted(parts):
        p = parts[seq]
        if p["call"] < a.from_call or shown >= a.parts:
            continue
        shown += 1
        print("%6d %5d %3s %10.1f %7.1f %9.3f %9.3f %9.3f %9.3f" % (
            seq, p["call"], "D2H" if p["down"] else "H2D", p["off"] / 2**20, p["nb"] / 2**20,
            p.get("T", -1), p.get("P", -1), p.get("D", -1), p.get("C", -1)))
    calls = defaultdict(list)
    for seq, p in parts.items():
        calls[p["call"]].append(p)
    print("\ncall  first-T  last-P  last-D  last-C  (ms)")
    for c in sorted(calls):
        ps = calls[c]
        print("%4d %8.3f %7.3f %7.3f %7.3f" % (c, min(p.get("T", 1e9) for p in ps), max(p.get("P", -1) for p in ps),
                                              max(p.get("D", -1) for p in ps), max(p.get("C", -1) for p in ps)))
    print("\n%d waits for room; first 40 (ms, oldest part):" % len(waits))
    print(" ".join("%.3f@%d" % w for w in waits[:40]))


if __name__ == "__main__":
    main()
