"""Square bf16 GEMM rate of hipBLASLt (torch.mm) on this device: the library ceiling the conv
kernels are compared with.  python tools/gemm_peak.py"""
import time

import torch

for n in (4096, 8192):
    a = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(n, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        a @ b
    torch.cuda.synchronize()
    t = time.time()
    for _ in range(20):
        a @ b
    torch.cuda.synchronize()
    dt = (time.time() - t) / 20
    print(f"{n}^3 bf16 GEMM: {2 * n ** 3 / dt / 1e12:.1f} TF/s", flush=True)
