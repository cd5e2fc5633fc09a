set -e
O=gpurun_out/r05g; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cut -c1-600 $O/bench.json
OUT=$O timeout -k 10 900 tools/config_sweep.sh > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
OUT=$O timeout -k 10 1200 tools/multirank_rehearsal.sh > $O/multirank.log 2>&1 || { tail -20 $O/multirank.log; exit 1; }
grep -h '"value"' $O/multirank/bench_gpus8.json | cut -c1-300
FRAMES=384 timeout -k 10 400 tools/ab_bench.sh 3 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_80v.so > $O/ab_80v.txt 2>&1 || { tail -20 $O/ab_80v.txt; exit 1; }
cat $O/ab_80v.txt
echo done
