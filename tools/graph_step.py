"""Eager vs HIP-graph replay of one full ResNet-50 training step (forward, CE loss, backward,
fused SGD + weight re-layout) on one GPU: shows how much of the eager step is host launch time.

python tools/graph_step.py [--batch 256] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from deep_vision_amd import ops as F
    from deep_vision_amd.models import ResNet50
    from deep_vision_amd.train.optim import FusedSGD

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = ResNet50().to(dev)
    opt = FusedSGD(model.parameters(), lr=0.1, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        opt.zero_grad()
        loss = F.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_eager = time.perf_counter() - t0
    print(f"eager: {t_eager / a.steps * 1e3:.2f} ms/step (host enqueue {t_enq / a.steps * 1e3:.2f} ms/step)", flush=True)

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        static_loss = step()
    torch.cuda.synchronize()
    losses = []
    for _ in range(3):
        g.replay()
        losses.append(float(static_loss.item()))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        g.replay()
    torch.cuda.synchronize()
    t_graph = time.perf_counter() - t0
    print(f"graph: {t_graph / a.steps * 1e3:.2f} ms/step  ({a.batch * a.steps / t_graph:.0f} img/s) losses {losses}",
          flush=True)


if __name__ == "__main__":
    main()
