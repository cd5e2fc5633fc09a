set -e
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MIPGPU_SLOT_EVENTS=nofence timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pipeline or async or per_frame or ticket or pageable or decisions or contract or dropped or stress" > $O/pytest_nofence.log 2>&1 || { tail -30 $O/pytest_nofence.log; exit 1; }
tail -2 $O/pytest_nofence.log
for i in 1 2 3; do MIPGPU_SLOT_EVENTS=nofence timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "stress or per_frame" > $O/stress_$i.log 2>&1 || { tail -30 $O/stress_$i.log; exit 1; }; tail -1 $O/stress_$i.log; done
echo done
