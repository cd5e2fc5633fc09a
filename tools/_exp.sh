set -e
cd /root/repo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
for lib in filt0 filt1; do MIPGPU_LIB=$PWD/abtest/$lib.so timeout -k 10 120 python tools/filter_bench.py > gpurun_out/fb_$lib.json 2>/dev/null; done
python - <<'PY'
import json
for lib in ("filt0","filt1"):
    d=json.load(open("gpurun_out/fb_%s.json"%lib))
    print(lib, {k[12:]: v["ms_per_launch"] for k,v in d["filters"].items()}, d.get("copy_calibration"))
PY
