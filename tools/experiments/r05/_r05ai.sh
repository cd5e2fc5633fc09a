set -e
O=gpurun_out/r05ai; mkdir -p $O
export TMPDIR=/tmp
rm -rf /tmp/pt
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/pt -o t --output-format csv -- python -u tools/e2e_probe.py --reps 2 --calls 1 128:dec:pinned:mb=384 > $O/rates.jsonl 2> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 tools/trace_timeline.py /tmp/pt --last 40 > $O/timeline.txt
cat $O/rates.jsonl | cut -c1-300
echo done
