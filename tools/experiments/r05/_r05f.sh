set -e
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pipeline or async or per_frame or ticket or pageable or decisions or contract or dropped or stress or many_launches or small_launch" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F5=filterFrame_2d_float_5x5_quarterCtu
C="1:dec:pinned 1:full:pinned 2:dec:pinned:$F5:2"
for v in default noext nofence; do
  case $v in default) E="";; noext) E="MIPGPU_EXT_DONE=0";; nofence) E="MIPGPU_SLOT_EVENTS=nofence";; esac
  env $E timeout -k 10 200 python -u tools/e2e_probe.py --reps 7 $C | sed "s/^/$v /" | cut -c1-400 | tee -a $O/rates.txt
done
FRAMES=384 timeout -k 10 300 tools/ab_bench.sh 3 vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_6w.so tools/bin/lib_80v.so 2>&1 | tee $O/ab_6w.txt
echo done
