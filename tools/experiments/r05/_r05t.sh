set -e
F5=filterFrame_2d_float_5x5_quarterCtu
OUT=gpurun_out/r05t MIPGPU_STAGE_STATS=1 bash tools/pipeline_probe.sh 1:dec:pageable 2:full:pinned:$F5:2 2:full:pageable:$F5:2 1:full:pageable
python3 tools/trace_timeline.py /tmp/pipe_trace --last 120 > gpurun_out/r05t/timeline_long.txt
