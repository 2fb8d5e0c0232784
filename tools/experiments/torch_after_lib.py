"""Does torch see the GPU after libflodbadd_gpu.so initialised HIP in the same process?"""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
order = sys.argv[1] if len(sys.argv) > 1 else "lib-first"
if order == "torch-first":
    import torch
    print("torch first:", torch.cuda.is_available(), torch.cuda.device_count(), flush=True)
from flodbadd_amd import _native as N
print("lib devices:", N.device_count(), flush=True)
import torch
print("torch after lib:", torch.cuda.is_available(), torch.cuda.device_count(), os.environ.get("HIP_VISIBLE_DEVICES"), os.environ.get("ROCR_VISIBLE_DEVICES"), os.environ.get("CUDA_VISIBLE_DEVICES"), flush=True)
