#!/bin/bash
env | grep -E "^(HIP|HSA|ROC|AMD|GPU|CUDA)" | sort
cat /sys/module/amdgpu/version 2>/dev/null; cat /proc/driver/amdgpu/version 2>/dev/null
python3 - <<'PY'
import ctypes, torch, time
torch.cuda.init()
s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
x = torch.randn(4096, 4096, device='cuda')
s.record(); y = x @ x; e.record(); torch.cuda.synchronize()
print("torch event ms", s.elapsed_time(e))
PY
timeout -k 10 200 python scripts/dbg_stats.py
