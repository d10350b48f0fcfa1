"""Diagnostic (GPU): the library GEMM rate (torch.matmul -> hipBLASLt) on the ViT-B/14 block shapes
(batch 128 at 336 x 336: M = 128 * 577 rows), for comparison with the modality engine's own
`gemm_tile_kernel`.   python tools/gemm_probe.py [batch]
"""
import sys

import torch

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
M = B * 577
dev = torch.device("cuda", 0)
for name, K, N in (("qkv", 768, 2304), ("out", 768, 768), ("fc1", 768, 3072), ("fc2", 3072, 768)):
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
    bias = torch.randn(N, device=dev, dtype=torch.bfloat16)
    for label, fn in (("mm", lambda: a @ w.t()), ("addmm", lambda: torch.addmm(bias, a, w.t()))):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) * 1e3 / reps
        tf = 2.0 * M * N * K / us / 1e6
        print(f"{name:4s} {label:6s} M={M} N={N} K={K}: {us:8.1f} us  {tf:7.1f} TFLOP/s  ({tf / 2500:.2f} of peak)",
              flush=True)
