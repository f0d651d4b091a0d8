#!/bin/bash
# RCCL one-rank init next to torch's runtime (diagnostics)
out=gpurun_out/r04rccl; mkdir -p $out
timeout -k 10 120 python -u -c "
from opentsdb_amd import engine as E
print('lib count', E.device_count())
e = E.Engine(devices=[0], transport=E.MD_RCCL); print('rccl ok before torch'); e.close()
import torch; print('torch count', torch.cuda.device_count())
try:
    e = E.Engine(devices=[0], transport=E.MD_RCCL); print('rccl ok after torch count'); e.close()
except Exception as ex: print('rccl FAILS after torch count:', ex)
" 2>&1 | tail -8
timeout -k 10 300 python -u -m pytest tests/test_gpu_multidev.py -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
echo rc=$?; tail -3 $out/pytest.log
