import json, sys
for l in sys.stdin:
    d = json.loads(l)
    r = sorted(d["fps_all"])
    out = {"AMD_DIRECT_DISPATCH": int(sys.argv[1]), "MIPGPU_MERGE": int(sys.argv[2]), "case": d["case"], "calls": d["calls"],
           "median": d["fps"], "best": r[-1], "p25": r[len(r) // 4], "rounds": d["fps_all"], "host_stats": d["host_stats"]}
    print(json.dumps(out))
