"""Roofline of one ResNet-50 V1 bf16 training step (batch 256) on MI355X.

Per conv: fwd / dgrad / wgrad FLOPs and the minimum HBM bytes (read operands once, write the
result once, bf16 activations). Per BN: the passes the current design makes. Prints the
compute-bound and memory-bound floors with practical ceilings (1.3 PF/s MFMA bf16 for a
well-pipelined HIP GEMM, 5.5 TB/s streaming) so measured kernel times can be read as a
fraction of speed-of-light.

usage: python tools/roofline.py [batch]
"""
import sys

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
PF = 1.3e15
BW = 5.5e12


def layers():
    out = [("stem", 3, 64, 224, 7, 2)]
    cin, h = 64, 56
    for planes, blocks, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
        for b in range(blocks):
            s = stride if b == 0 else 1
            ho = h // s
            out.append((f"{planes}.{b}.c1", cin, planes, h, 1, s))       # V1: stride on the first 1x1
            out.append((f"{planes}.{b}.c2", planes, planes, ho, 3, 1))
            out.append((f"{planes}.{b}.c3", planes, planes * 4, ho, 1, 1))
            if b == 0:
                out.append((f"{planes}.{b}.proj", cin, planes * 4, h, 1, s))
            cin, h = planes * 4, ho
    return out


tot = {"flop": 0.0, "t_c": 0.0, "t_m": 0.0, "t": 0.0, "bytes": 0.0}
print(f"{'layer':14s} {'GF':>8s} {'MB in':>8s} {'MB out':>8s} {'floor us (fwd/dgrad/wgrad)':>30s}")
for name, ci, co, h, k, s in layers():
    ho = (h + 2 * (k // 2) - k) // s + 1
    m = B * ho * ho
    flop = 2.0 * m * co * ci * k * k
    xin = B * h * h * ci * 2
    yout = m * co * 2
    w = co * ci * k * k * 2
    ts = []
    for kind, rd, wr in (("fwd", xin + w, yout), ("dgrad", yout + w, xin), ("wgrad", xin + yout, w * 2)):
        tc, tm = flop / PF, (rd + wr) / BW
        ts.append(max(tc, tm))
        tot["flop"] += flop
        tot["t_c"] += tc
        tot["t_m"] += tm
        tot["t"] += max(tc, tm)
        tot["bytes"] += rd + wr
    print(f"{name:14s} {flop / 1e9:8.1f} {xin / 1e6:8.1f} {yout / 1e6:8.1f}   " + " / ".join(f"{t * 1e6:7.1f}" for t in ts))

# BatchNorm + activation traffic (elements of every BN output); stats fused in the conv epilogue
bn_elems = 0
for name, ci, co, h, k, s in layers():
    ho = (h + 2 * (k // 2) - k) // s + 1
    bn_elems += B * ho * ho * co
bn_fwd = bn_elems * 2 * 2            # apply: read z, write a
bn_bwd = bn_elems * 2 * 5            # reduce: read g, z; apply: read g, z, write dz
print(f"\nconv: {tot['flop'] / 1e12:.2f} TFLOP, {tot['bytes'] / 1e9:.1f} GB min traffic")
print(f"conv floor: compute-only {tot['t_c'] * 1e3:.2f} ms, memory-only {tot['t_m'] * 1e3:.2f} ms, "
      f"per-kernel max {tot['t'] * 1e3:.2f} ms")
print(f"BN: {bn_elems / 1e9:.2f} G elements; fwd apply {bn_fwd / 1e9:.1f} GB = {bn_fwd / BW * 1e3:.2f} ms, "
      f"bwd {bn_bwd / 1e9:.1f} GB = {bn_bwd / BW * 1e3:.2f} ms")
step = tot["t"] + (bn_fwd + bn_bwd) / BW
print(f"step floor (unfused BN passes) {step * 1e3:.2f} ms -> {B / step:.0f} img/s")
