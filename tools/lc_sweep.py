import sys; sys.path.insert(0,'tools')
from loss_curve import run_curve
for name in ("resnet50","mobilenet1"):
  for lr, noise in ((0.05,1.0),(0.02,1.0),(0.02,0.3),(0.01,0.3)):
    c=run_curve(name,bs=64,steps=100,lr=lr,noise=noise)
    for k,v in c.items(): print(name,lr,noise,k,v[::10],v[-1],flush=True)
