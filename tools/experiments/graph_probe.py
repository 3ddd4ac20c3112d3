"""Probe: the ViT-B b256 forward eager vs replayed from a captured HIP graph (torch.cuda.CUDAGraph over the
C-ABI launches). Prints ms per step for both and whether the logits match. Diagnostic only."""
import sys, time
sys.path.insert(0, ".")
import torch
from quantized_vit_amd import _lib
from quantized_vit_amd.calibrate import build_quantized_vit, synthetic_images

_lib.load()
dev = torch.device("cuda", 0)
model = build_quantized_vit("vit_base_patch16_224", seed=0, device=dev)
x = synthetic_images(256, 224, seed=1000, device=dev)
steps = 20
with torch.no_grad():
    for _ in range(3):
        y0 = model(x)
    torch.cuda.synchronize()
    def eager():
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(steps):
            model(x)
        torch.cuda.synchronize(); return (time.perf_counter() - t) / steps * 1e3
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            model(x)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        yg = model(x)
    torch.cuda.synchronize()
    def replay():
        torch.cuda.synchronize(); t = time.perf_counter()
        for _ in range(steps):
            g.replay()
        torch.cuda.synchronize(); return (time.perf_counter() - t) / steps * 1e3
    g.replay(); torch.cuda.synchronize()
    print("logits equal:", bool(torch.equal(yg, y0)), flush=True)
    for r in range(3):
        e, gr = eager(), replay()
        print(f"round {r}: eager {e:.3f} ms  graph {gr:.3f} ms  ({(e - gr) / e * 100:+.2f} %)", flush=True)
