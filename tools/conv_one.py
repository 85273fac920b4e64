"""Run one conv pass repeatedly (for rocprofv3 counter collection)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from deep_vision_amd.ops import conv as C
from deep_vision_amd.ops.common import as_nhwc
cin, cout, H, R, st, pd = [int(v) for v in sys.argv[1:7]]
mode = sys.argv[7] if len(sys.argv) > 7 else "fwd"
N = int(os.environ.get("BATCH", "256"))
x = as_nhwc(torch.randn(N, cin, H, H, device="cuda"))
w = torch.randn(cout, cin, R, R, device="cuda") * 0.05
y = C.conv2d(x, w, None, st, pd)
dy = torch.randn_like(y.float()).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
Cg = C._gather_channels(x, cin, 1)
for _ in range(5):
    if mode == "fwd":
        C.conv2d(x, w, None, st, pd)
    elif mode == "dgrad":
        C._dgrad(dy, w, x.shape, Cg, 1, (st, st), (pd, pd), (1, 1), x.device)
    else:
        C._wgrad(x, dy, w, Cg, 1, (st, st), (pd, pd), (1, 1))
torch.cuda.synchronize()
