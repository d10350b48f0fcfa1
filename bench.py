"""Headline benchmark: in-context rows/sec on PAD-UFES-20-shaped inputs (BASELINE.json).

Workload (config C): N = 1838 support + Q = 460 query rows, F = 21
features (18 categorical + 3 numeric), one 768-d image embedding per row, MGM (64
heads) + CAP (24 queries) mixer, 12-layer E=192 PerFeatureTransformer, 4 ensemble
members per GPU (feature-shuffle + class-permutation members as EnsembleConfig
builds them), synthetic data and random-init weights of that architecture.

One step = one ``predict_proba`` pass of the hot path with inputs resident in HBM:
mixer once (the image is identical for every member), 4 member forwards per GPU,
one RCCL all-gather of the per-member logits, ensemble softmax-mean.  ``value`` =
sum over members of (N + Q) / wall time, aggregated over all ranks (weak scaling:
4 members per GPU).  Launch with ``torchrun --nproc-per-node N bench.py --gpus N``
for N > 1.

Also reported: ``roofline`` of the dominant kernel (sample-axis attention, bf16
MFMA; algorithmic flops 4*T*Nq*Nk*E per launch; every launch inside the timed region
bracketed by HIP events on its lane stream, mmpfn_kernel_timing) and ``cpu_baseline`` (the oracle's CPU restatement of the same
forward -- the reference's torch-SDPA branch -- on the host cores, bounded sample).
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests" / "golden"))

METRIC = "in-context rows/sec (support+query), PAD-UFES-20 shape, 1/2/4/8 MI355X"
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
HBM_PEAK_GBS = 8000.0

S_ROWS, N_TRAIN, N_FEAT, N_CAT, N_CLASSES = 2298, 1838, 21, 18, 6
MGM, CAP, MEMBERS_PER_GPU = 64, 24, 4


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--precision", choices=["bf16", "f32"], default="bf16")
    p.add_argument("--members", type=int, default=MEMBERS_PER_GPU, help="members per GPU")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--attn-reps", type=int, default=20)
    p.add_argument("--lanes", type=int, default=None, help="concurrent member lanes per GPU (default: engine's)")
    p.add_argument("--batch", type=int, default=None, help="members per batched forward (default: engine's)")
    p.add_argument("--api-steps", type=int, default=3, help="timed predict_proba calls of the API leg (0: skip)")
    p.add_argument("--no-kv-cache", dest="kv_cache", action="store_false", help="skip the fit_with_cache leg")
    return p.parse_args()


def build_workload(device, world, members_per_gpu):
    from synth import synth_image, synth_labels, synth_state_dict, synth_table

    from multimodalpfn_amd.model.spec import ModelConfig, state_dict_spec
    from multimodalpfn_amd.model.transformer import PerFeatureTransformer

    cfg = ModelConfig(mgm_heads=MGM, cap_heads=CAP)
    sd = synth_state_dict(state_dict_spec(cfg), 2)
    model = PerFeatureTransformer(cfg)
    model.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
    norm = next(e for e in model.encoder if "InputNormalizationEncoderStep" in str(e.__class__))
    norm.remove_outliers, norm.remove_outliers_sigma = True, 12.0  # classifier.fit (classifier.py:396-406)
    model.to(device)
    x = synth_table(S_ROWS, N_FEAT, 2, n_cat=N_CAT)
    y = synth_labels(S_ROWS, N_CLASSES, 2)
    image = synth_image(S_ROWS, 1, 2)
    M = members_per_gpu * world
    rng = np.random.default_rng(0)
    members = []
    for m in range(M):
        fperm = rng.permutation(N_FEAT)  # ShuffleFeaturesStep
        cperm = rng.permutation(N_CLASSES)  # class_permutation
        xm = torch.from_numpy(np.ascontiguousarray(x[:, fperm])).to(device)
        ym = cperm[y[:N_TRAIN].astype(np.int64)].astype(np.float32)
        members.append((xm, ym, np.argsort(cperm)))
    return cfg, sd, model, x, y, image, members


def attn_traffic(T):
    """HBM bytes per attention launch over T token columns, from the committed PMC pass
    (tools/attn_pmc.sh: rocprofv3 FETCH_SIZE and WRITE_SIZE runs at that launch shape)."""
    H, d, S, N = 6, 32, S_ROWS, N_TRAIN
    for pmc in sorted((ROOT / "profiles" / "r01").glob("attn_item2_pmc*.json")):
        rec = json.loads(pmc.read_text())
        if rec.get("shape") == {"T": T, "H": H, "d": d, "S": S, "N": N}:
            return rec["hbm_bytes_per_launch"], str(pmc.relative_to(ROOT))
    return None, None


def live_roofline(lib, ctx, T_launch):
    """Roofline of the dominant kernel from the launches INSIDE the timed region: HIP events
    recorded by the engine on each lane's stream around every attn_item2 launch."""
    import ctypes

    ms, n, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    assert lib.mmpfn_kernel_timing_read(ctx, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(fl)) == 0
    if n.value == 0:
        return None
    H, d, S, N = 6, 32, S_ROWS, N_TRAIN
    per_ms, per_fl = ms.value / n.value, fl.value / n.value
    uniform = abs(per_fl - 4.0 * T_launch * S * N * H * d) < 1.0
    achieved = per_fl / (per_ms * 1e-3) / 1e12
    traffic, src = attn_traffic(T_launch) if uniform else (None, None)
    return {
        "bound": "mfma",
        "achieved": round(achieved, 1),
        "peak": BF16_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
        "traffic": traffic,
        "traffic_unit": f"HBM bytes per launch (PMC: 2 x FETCH_SIZE + WRITE_SIZE, {src})" if src else None,
        "algorithmic_bytes": 2 * T_launch * H * d * (S + 2 * N) + 2 * T_launch * S * H * d,
        "kernel": "attn_item2_kernel (sample-axis attention: train + test-MQA rows of one layer, all members "
                  "of a batched forward, per launch)",
        "launches_timed": n.value,
        "token_columns_per_launch": T_launch,
        "per_launch_ms": round(per_ms, 4),
        "per_launch_flop": per_fl,
        "timing": "HIP events on the launching lane stream around every launch in the timed region "
                  "(mmpfn_kernel_timing); lanes overlap, so a launch shares the GPU with the other lane's kernels",
    }


def time_item_attention(eng, T, reps, S=S_ROWS, N=N_TRAIN):
    """Average launch duration of the sample-axis attention kernel at the workload's shape.

    One launch = the whole attention-between-items of one layer (train rows on their own
    heads + test rows of all heads on head 0's K/V), HIP events on the engine stream."""
    H, d = 6, 32
    Q = S - N
    Npad = (N + 63) // 64 * 64
    dev = eng.device
    g = torch.Generator(device="cpu").manual_seed(0)
    q = torch.randn(T, H, S, d, generator=g).to(dev, torch.bfloat16)
    k = torch.randn(T, H, Npad, d, generator=g).to(dev, torch.bfloat16)
    vt = torch.randn(T, H, d, Npad, generator=g).to(dev, torch.bfloat16)
    o = torch.empty(T, S, H * d, device=dev, dtype=torch.bfloat16)
    lib, ctx = eng.lib, eng.ctx
    eng._bind_stream()
    stream = torch.cuda.current_stream(dev)

    def launch():
        rc = lib.mmpfn_item_attention_layer(ctx, q.data_ptr(), k.data_ptr(), vt.data_ptr(), o.data_ptr(), S, T, H,
                                            Npad, N)
        assert rc == 0, lib.mmpfn_last_error(ctx)

    for _ in range(3):
        launch()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch()
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    flops = 4.0 * T * (N + Q) * N * H * d  # train 4*T*N*N*E + test (MQA) 4*T*Q*N*E
    achieved = flops / (ms * 1e-3) / 1e12
    traffic, src = attn_traffic(T) if (S, N) == (S_ROWS, N_TRAIN) else (None, None)
    return {
        "bound": "mfma",
        "achieved": round(achieved, 1),
        "peak": BF16_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
        "traffic": traffic,
        "traffic_unit": f"HBM bytes per launch (PMC: 2 x FETCH_SIZE + WRITE_SIZE, {src})" if src else None,
        "algorithmic_bytes": 2 * T * H * d * (S + 2 * N) + 2 * T * S * H * d,
        "kernel": "attn_item2_kernel (sample-axis attention, train + test-MQA rows of one layer per launch)",
        "per_launch_ms": round(ms, 4),
        "per_launch_flop": flops,
    }


def forward_flops(T, S=S_ROWS, N=N_TRAIN, E=192, FF=768, L=12) -> float:
    """Algorithmic flops of one member forward's layer stack:
    feature attention (QKV, T x T attention, out-projection), item attention (Q of all rows,
    K/V of the train rows, train + test-MQA attention, out-projection) and the MLP."""
    Q = S - N
    feat = 2 * S * T * E * 3 * E + 4 * S * T * T * E + 2 * S * T * E * E
    item = 2 * S * T * E * E + 2 * N * T * E * 2 * E + 4 * T * N * N * E + 4 * T * Q * N * E + 2 * S * T * E * E
    mlp = 4 * S * T * E * FF
    return float(L * (feat + item + mlp))


def mixer_flops(S=S_ROWS, D=768, E=192, mgm=MGM, cap=CAP) -> float:
    """MGM (per head Linear(768,768) + Linear(384,192)) and CAP (K|V projection of the
    mgm tokens, attention, out-projection, FFN) of one predict (A7-A8)."""
    mg = 2 * S * mgm * (D * D + (D // 2) * E)
    cp = 2 * S * mgm * E * 2 * E + 4 * S * cap * mgm * E + 2 * S * cap * (E * E + E * 2 * E + 2 * E * E)
    return float(mg + cp)


def kv_cache_leg(eng, members, img, prec, steps):
    """``fit_mode="fit_with_cache"`` serving rate: each member's train rows forwarded once
    (cache build, timed separately), then every predict forwards only the Q test rows of each
    member against its cached head-0 K/V (mmpfn_cache_predict).  Not the headline metric."""
    N, Q = N_TRAIN, S_ROWS - N_TRAIN
    tok = eng.mixer_tokens(img, prec)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    caches = [eng.cache_build(xm[:N], tok[:N], ym, prec) for xm, ym, _ in members]
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0

    def predict():
        tq = eng.mixer_tokens(img[N:], prec)
        return eng.cache_predict_many(caches, [xm[N:] for xm, _, _ in members], tq)

    predict()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        predict()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    out = {
        "query_rows_per_s": round(len(members) * Q / dt, 1),
        "ms_per_predict": round(dt * 1e3, 3),
        "ms_cache_build_all_members": round(t_build * 1e3, 3),
        "cache_bytes_per_member": caches[0].nbytes,
        "note": "fit_with_cache: Q test rows per member against the device-resident train-KV cache",
    }
    for c in caches:
        c.free()
    return out


def cpu_baseline(sd, x, y, image):
    """Oracle (CPU restatement of the reference forward, SDPA branch) on one member."""
    from multimodalpfn_amd.model.spec import ModelConfig
    from oracle.forward import OracleSpec, oracle_forward

    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    cfg = ModelConfig(mgm_heads=MGM, cap_heads=CAP)
    spec = OracleSpec(mgm_heads=cfg.mgm_heads, cap_heads=cfg.cap_heads)
    w = {k: torch.from_numpy(v) for k, v in sd.items()}
    args = (spec, w, torch.from_numpy(x), torch.from_numpy(image), torch.from_numpy(y[:N_TRAIN]))
    t0 = time.perf_counter()
    oracle_forward(*args, use_sdpa=True)
    dt = time.perf_counter() - t0
    return {
        "value": round(S_ROWS / dt, 2),
        "unit": "rows/s",
        "cores": threads,
        "kind": "port",
        "sample": f"1 member forward of config C (S={S_ROWS}, 12 layers, MGM64+CAP24, fp32, torch SDPA "
                  f"branch) on {threads} host threads: {dt:.1f} s",
    }


def api_end_to_end(cfg, sd, x, y, image, n_estimators, prec_f32, steps, world):
    """``MMPFNClassifier.predict_proba`` wall time from host numpy inputs (PCIe-inclusive).

    run.py's interface config (no preprocessing, no fingerprint), the 18 categorical
    columns marked, ``n_estimators`` members (sharded over ranks when distributed).
    """
    import tempfile

    import torch.distributed as dist

    from multimodalpfn_amd import MMPFNClassifier
    from multimodalpfn_amd.constants import ModelInterfaceConfig
    from multimodalpfn_amd.preprocessing import PreprocessorConfig
    from api_cases import ckpt_config

    with tempfile.TemporaryDirectory() as tmp:
        ck = Path(tmp) / "mmpfn_configC.ckpt"
        torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}, "config": ckpt_config(cfg)}, ck)
        clf = MMPFNClassifier(
            model_path=str(ck), mixer_type="MGM+CAP", mgm_heads=MGM, cap_heads=CAP, features_per_group=2,
            n_estimators=n_estimators, categorical_features_indices=list(range(N_CAT)),
            ignore_pretraining_limits=True, inference_precision=torch.float32 if prec_f32 else "auto",
            inference_config=ModelInterfaceConfig(FINGERPRINT_FEATURE=False,
                                                  PREPROCESS_TRANSFORMS=[PreprocessorConfig(name="none")]),
        )
        X = x.astype(np.float64)
        labels = y.astype(np.int64)
        clf.fit(X[:N_TRAIN], image[:N_TRAIN], labels[:N_TRAIN])
    Xq, imq = X[N_TRAIN:], image[N_TRAIN:]
    clf.predict_proba(Xq, imq)  # warm-up (engine build, weight upload)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        proba = clf.predict_proba(Xq, imq)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    assert np.isfinite(proba).all()
    return {
        "value": round(n_estimators * S_ROWS * steps / dt, 1),
        "unit": "rows/s",
        "ms_per_predict": round(dt / steps * 1e3, 3),
        "members": n_estimators,
        "note": "MMPFNClassifier.predict_proba on host numpy inputs: validation + per-member host transform, "
                "H2D copies, mixer, member forwards, aggregation, D2H (PCIe-inclusive; not the headline value)",
    }


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    from multimodalpfn_amd import _lib
    from multimodalpfn_amd.parallel import allgather_logits, lpt_assign

    prec = _lib.PREC_BF16 if args.precision == "bf16" else _lib.PREC_F32
    cfg, sd, model, x, y, image, members = build_workload(device, world, args.members)
    eng = model.engine(device)
    img = torch.from_numpy(image).to(device)
    M = len(members)
    T = (N_FEAT + 1) // 2 + CAP + 1
    assignment = lpt_assign([float(T * S_ROWS * N_TRAIN)] * M, world)
    mine = assignment[rank]
    perms = np.stack([members[m][2] for m in range(M)])

    def step():
        tokens = eng.mixer_tokens(img, prec)
        outs = eng.forward_many([(members[m][0], tokens, members[m][1]) for m in mine], prec, args.lanes,
                                args.batch)
        local = torch.stack(outs)
        allm = allgather_logits(local, assignment, rank)
        return eng.aggregate(allm, perms, N_CLASSES, 0.9, False)

    probs = step()
    eng.status()  # NaN check once (reference raises ValueError)
    assert torch.isfinite(probs).all()
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.lib.mmpfn_kernel_timing(eng.ctx, 1)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.lib.mmpfn_kernel_timing(eng.ctx, 0)
    batch = eng.batch if args.batch is None else args.batch
    live = live_roofline(eng.lib, eng.ctx, T * min(batch, len(mine))) if rank == 0 else None
    if world > 1:
        tt = torch.tensor([dt], device=device, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
    rows = M * S_ROWS * args.steps
    value = rows / dt
    step_flop = len(mine) * forward_flops(T) + mixer_flops()  # per rank
    wf = step_flop * args.steps / dt / 1e12  # TFLOP/s of one rank (its wall time is the job's max)

    api = None
    if args.api_steps > 0:
        try:
            api = api_end_to_end(cfg, sd, x, y, image, M, prec == _lib.PREC_F32, args.api_steps, world)
        except Exception as e:  # noqa: BLE001 - reported, the headline number stands on its own
            api = {"error": f"{type(e).__name__}: {e}"}
    kv = kv_cache_leg(eng, [members[m] for m in mine], img, prec, args.steps) if args.kv_cache and mine else None
    roof = None
    if rank == 0:
        iso = time_item_attention(eng, T, args.attn_reps)
        roof = live if live is not None else iso
        roof["isolated_single_member_launch"] = {k: iso[k] for k in ("achieved", "frac", "per_launch_ms", "traffic")}
        if live is not None and live["token_columns_per_launch"] != T:  # the step's launch shape, alone
            isb = time_item_attention(eng, live["token_columns_per_launch"], args.attn_reps)
            roof["isolated_same_shape_launch"] = {k: isb[k] for k in ("achieved", "frac", "per_launch_ms", "traffic")}
        # the same kernel at BASELINE.json's other single-GPU shapes (one layer's launch, alone):
        # B = 4096 support x 100 features (G = 50, T = 51), E = 10k support rows (G = 10, T = 11)
        roof["other_configs_isolated_launch"] = {}
        for name, (Tc, Sc, Nc) in {"B: S=5120 N=4096 T=51": (51, 5120, 4096),
                                   "E: S=12000 N=10000 T=11": (11, 12000, 10000)}.items():
            r = time_item_attention(eng, Tc, max(3, args.attn_reps // 4), Sc, Nc)
            roof["other_configs_isolated_launch"][name] = {k: r[k] for k in ("achieved", "frac", "per_launch_ms")}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(sd, x, y, image)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "rows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if prec == _lib.PREC_BF16 else "f32",
            "data": "synthetic (PAD-UFES-20 shape; random-init weights of the MMPFN architecture)",
            "config": {
                "workload": "config C: PAD-UFES-20 image+tabular, N=1838 support + Q=460 query rows, F=21 "
                            "(18 cat + 3 num), image [S,1,768], MGM 64 heads + CAP 24, 12 layers E=192",
                "members_per_gpu": args.members,
                "lanes": eng.lanes if args.lanes is None else args.lanes,
                "members_per_batched_forward": eng.batch if args.batch is None else args.batch,
                "members_total": M,
                "rows_per_member": S_ROWS,
                "tokens_per_row": T,
                "parallelism": f"ensemble members sharded over {world} GPU(s) + RCCL all-gather of logits",
            },
            "roofline": roof,
            "whole_forward": {
                "tflop_per_step_per_gpu": round(step_flop / 1e12, 3),
                "achieved": round(wf, 1),
                "unit": "TFLOP/s per GPU",
                "frac": round(wf / BF16_PEAK_TFLOPS, 4),
                "note": "algorithmic flops of the mixer + every member's 12-layer stack (SURVEY.md 8d) / step time",
            },
            "cpu_baseline": cpu,
            "api_end_to_end": api,
            "kv_cache_predict": kv,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
