"""Diagnostic (GPU): where predict_proba's wall time goes beyond the device forward at config C.

Run under `rocprofv3 --kernel-trace` (tools/api_gaps.sh), it makes the classifier of bench.py's api leg (run.py's
interface config), runs 3 + 10 predicts, then `python3 tools/api_gaps.py --trace <run_kernel_trace.csv>` splits the
trace into predicts at the mixer's first kernel and prints per predict: the span of its kernels, the GPU-busy time
inside it, the idle gaps > 20 us with the kernels either side, and the gap to the next predict's first kernel."""
import csv
import sys
import time
from pathlib import Path


def analyse(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    first = [i for i, r in enumerate(rows) if "ln_rows_kernel" in r["Kernel_Name"]]
    # a predict's mixer starts with the image LayerNorm; keep the last 10 predicts
    starts = first[-10:]
    ends = starts[1:] + [len(rows)]
    prev_end = None
    tot = {"span": 0, "busy": 0, "between": 0}
    for k, (a, b) in enumerate(zip(starts, ends)):
        ks = rows[a:b]
        t0, t1 = int(ks[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in ks)
        busy, ce, cs, gaps, prev = 0, None, None, [], None
        for r in ks:
            s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            if ce is None:
                cs, ce, prev = s, e, r
                continue
            if s > ce:
                busy += ce - cs
                gaps.append((s - ce, prev["Kernel_Name"][:48], r["Kernel_Name"][:48]))
                cs = s
            if e > ce:
                ce, prev = e, r
        busy += ce - cs
        between = (t0 - prev_end) if prev_end is not None else 0
        prev_end = t1
        if k:
            tot["span"] += t1 - t0
            tot["busy"] += busy
            tot["between"] += between
        print(f"predict {k}: span {(t1 - t0) / 1e6:.3f} ms, busy {busy / 1e6:.3f} ms, idle inside "
              f"{(t1 - t0 - busy) / 1e6:.3f} ms, gap before {between / 1e6:.3f} ms, kernels {len(ks)}")
        for g, p, n in sorted(gaps, reverse=True)[:6]:
            if g > 20000:
                print(f"    {g / 1e3:8.1f} us  {p}  ->  {n}")
    n = len(starts) - 1
    print(f"mean over predicts 1..{n}: span {tot['span'] / n / 1e6:.3f} ms, busy {tot['busy'] / n / 1e6:.3f} ms, "
          f"gap between predicts {tot['between'] / n / 1e6:.3f} ms")


def run():
    import numpy as np
    import torch

    root = Path(__file__).resolve().parent.parent
    sys.path[:0] = [str(root), str(root / "tests" / "golden")]
    import tempfile

    import bench
    from api_cases import ckpt_config

    from multimodalpfn_amd import MMPFNClassifier
    from multimodalpfn_amd.constants import ModelInterfaceConfig
    from multimodalpfn_amd.preprocessing import PreprocessorConfig

    cfg, sd, model, x, y, image, members = bench.build_workload(torch.device("cuda", 0), 1, 4)
    with tempfile.TemporaryDirectory() as tmp:
        ck = Path(tmp) / "c.ckpt"
        torch.save({"state_dict": {k: torch.from_numpy(v) for k, v in sd.items()}, "config": ckpt_config(cfg)}, ck)
        clf = MMPFNClassifier(model_path=str(ck), mixer_type="MGM+CAP", mgm_heads=64, cap_heads=24,
                              features_per_group=2, n_estimators=4, categorical_features_indices=list(range(18)),
                              ignore_pretraining_limits=True,
                              inference_config=ModelInterfaceConfig(FINGERPRINT_FEATURE=False, PREPROCESS_TRANSFORMS=[
                                  PreprocessorConfig(name="none")]))
        X = x.astype(np.float64)
        clf.fit(X[:1838], image[:1838], y[:1838].astype(np.int64))
    Xq, imq = X[1838:], image[1838:]
    for _ in range(3):
        clf.predict_proba(Xq, imq)
    t0 = time.perf_counter()
    for _ in range(10):
        clf.predict_proba(Xq, imq)
    print("ms per predict", (time.perf_counter() - t0) * 100)
    host_timeline(clf, Xq, imq)


def host_timeline(clf, Xq, imq):
    """Host-side timeline of one predict: entry / exit times of the calls on the path (monkeypatched wrappers)."""
    import multimodalpfn_amd.classifier as C
    import multimodalpfn_amd.engine as E
    import multimodalpfn_amd.inference as I

    ev = []
    T0 = [0.0]

    def wrap(owner, name, label):
        f = getattr(owner, name)

        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                ev.append((t - T0[0], time.perf_counter() - T0[0], label))
        setattr(owner, name, g)
        return f

    saved = [(E.HipEngine, n, wrap(E.HipEngine, n, n)) for n in
             ("mixer_tokens", "forward_batch", "forward", "status", "aggregate", "_prepare", "_pos")]
    saved += [(I, "_h2d", wrap(I, "_h2d", "_h2d")), (I, "_mixer_tokens", wrap(I, "_mixer_tokens", "_mixer_tokens"))]
    saved += [(C.MMPFNClassifier, "_encode_predict_X", wrap(C.MMPFNClassifier, "_encode_predict_X", "encode_X"))]
    pre = clf.executor_.preprocessors[0].__class__
    saved += [(pre, "transform", wrap(pre, "transform", "member_transform"))]
    for _ in range(2):
        ev.clear()
        T0[0] = time.perf_counter()
        clf.predict_proba(Xq, imq)
        tend = time.perf_counter() - T0[0]
    for a, b, lab in sorted(ev):
        print(f"  host {a * 1e3:8.3f} -> {b * 1e3:8.3f} ms  {lab}")
    print(f"  host predict_proba returns at {tend * 1e3:.3f} ms")
    for owner, n, f in saved:
        setattr(owner, n, f)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--trace"]:
        analyse(sys.argv[2])
    else:
        run()
