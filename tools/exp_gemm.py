"""Time torch fp32 / bf16 matmul at the layers' post-aggregate GEMM shapes (measurement helper)."""
import json
import torch

dev = torch.device("cuda:0")
res = []
for m, k, n in ((10_000_000, 256, 256), (10_000_000, 128, 128), (2_449_029, 100, 100), (1_000_000, 128, 128)):
    for dt in (torch.float32, torch.bfloat16):
        x = torch.randn(m, k, device=dev, dtype=dt)
        w = torch.randn(k, n, device=dev, dtype=dt)
        b = torch.randn(n, device=dev, dtype=dt)
        for _ in range(3):
            torch.addmm(b, x, w)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            torch.addmm(b, x, w)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        byt = (m * k + m * n) * x.element_size()
        res.append(dict(m=m, k=k, n=n, dtype=str(dt), ms=round(ms, 3), tflops=round(2 * m * k * n / ms / 1e9, 1),
                        tbps=round(byt / ms / 1e9, 2)))
        print(json.dumps(res[-1]), flush=True)
        del x, w, b
