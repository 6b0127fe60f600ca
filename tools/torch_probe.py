import os, subprocess
print({k: v for k, v in os.environ.items() if any(s in k for s in ("HIP", "ROCR", "HSA", "CUDA", "GPU", "LD_"))})
import torch
print("torch", torch.__version__, "hip", torch.version.hip)
try:
    print("count", torch._C._cuda_getDeviceCount())
except Exception as e:
    print("getDeviceCount error", e)
print("avail", torch.cuda.is_available())
try:
    torch.zeros(1).cuda()
except Exception as e:
    print("cuda() error:", e)
