"""Diagnostic (GPU): time / profile the modality towers (DINOv2 ViT-B/14 at 336 x 336, ELECTRA-base).

python tools/modality_prof.py [vit|text] [bf16|f32] [batch]   (run under rocprofv3 --kernel-trace --stats)
"""
import sys
import time
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "tests" / "golden")]
import bench  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "vit"
prec = sys.argv[2] if len(sys.argv) > 2 else "bf16"
B = int(sys.argv[3]) if len(sys.argv) > 3 else 128
dev = torch.device("cuda", 0)
if which == "vit":
    from modality_cases import vit_state
    from multimodalpfn_amd.modality import vit_base

    m = vit_base(patch_size=14, img_size=518, init_values=1.0, num_register_tokens=0, block_chunks=0, precision=prec)
    c = dict(dim=768, depth=12, heads=12, patch=14, img_size=518, init_values=1.0, offset=0.1, seed=31)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in vit_state(c).items()})
    x = torch.rand((B, 3, 336, 336), device=dev)
    run = lambda: m.cls_embeddings(x)  # noqa: E731
    fl = bench.vit_flops(B, 336, 336)
else:
    from modality_cases import text_config, text_state
    from multimodalpfn_amd.modality import ElectraTextEncoder

    tc = dict(vocab=30522, emb=768, dim=768, depth=12, heads=12, ffn=3072, max_pos=512, types=2, seed=32)
    m = ElectraTextEncoder(text_config(tc), precision=prec)
    m.load_state_dict({k: torch.from_numpy(v) for k, v in text_state(tc).items()})
    ids = torch.randint(1, 30522, (B, 128), device=dev)
    run = lambda: m.cls_embeddings(ids, torch.ones_like(ids))  # noqa: E731
    fl = 0.0
run()
torch.cuda.synchronize()
t0 = time.perf_counter()
import os  # noqa: E402
for _ in range(int(os.environ.get("ITERS", "5"))):
    run()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / int(os.environ.get("ITERS", "5"))
print(f"{which} {prec} B={B}: {dt * 1e3:.2f} ms per batch, {B / dt:.1f} items/s, {fl / dt / 1e12:.1f} TFLOP/s")
