"""Host-side native code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU).

``tests/native/host_check.cpp`` runs the engine's host code on the model's real shapes, built with
``g++ -fsanitize=address,undefined -fno-sanitize-recover=all``:
* the weight packing of ``mmpfn_finalize_weights`` (``csrc/weight_pack.h``): bf16 rounding, the out-projection
  transpose, the MLP K / hidden permutations, the feature-block LDS images, the LayerNorm fold;
* ``mmpfn_siphash24_rows`` (``csrc/host.cpp``), the fingerprint feature's row hash.
Any sanitizer report aborts the binary.  Its outputs are compared here with independent restatements
(numpy index arithmetic from the layouts the kernels document, torch's bf16 conversion, the numpy SipHash).
The GPU kernels cannot run under a sanitizer on this pool; this covers the C++ that runs on the host.
"""

from __future__ import annotations

import os
import shutil
import subprocess
from pathlib import Path

import numpy as np
import pytest
import torch

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "multimodalpfn_amd" / "csrc"
E, H, FH = 192, 6, 768
ST = 208  # FEAT_IMG_STRIDE


@pytest.fixture(scope="module")
def outputs(tmp_path_factory):
    gxx = shutil.which("g++")
    if gxx is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("host_check")
    exe = d / "host_check"
    cmd = [gxx, "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           "-fno-omit-frame-pointer", "-Wall", "-Werror", f"-I{CSRC}", str(ROOT / "tests/native/host_check.cpp"),
           str(CSRC / "host.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=300)
    # verify_asan_link_order=0: the environment may preload a library ahead of the ASan runtime
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), str(d)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "host_check ok" in r.stdout, r.stdout + r.stderr

    def load(name, dtype):
        return np.fromfile(d / name, dtype=dtype)

    return load


def test_f2bf_matches_torch(outputs):
    bits = outputs("f2bf_in.bin", np.uint32)
    mine = outputs("f2bf_out.bin", np.uint16)
    x = torch.from_numpy(bits.view(np.float32).copy())
    ref = x.to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16)
    nan = np.isnan(bits.view(np.float32))
    assert np.array_equal(mine[~nan], ref[~nan])
    # NaNs stay NaN (quiet, sign kept; torch returns one canonical NaN)
    assert np.all((mine[nan] & 0x7F80) == 0x7F80) and np.all((mine[nan] & 0x0040) != 0)
    assert np.array_equal(mine[nan] >> 15, (bits[nan] >> 31).astype(np.uint16))


def test_f2h_matches_torch(outputs):
    bits = outputs("f2bf_in.bin", np.uint32)
    mine = outputs("f2h_out.bin", np.uint16)
    x = torch.from_numpy(bits.view(np.float32).copy())
    ref = x.to(torch.float16).view(torch.int16).numpy().view(np.uint16)
    nan = np.isnan(bits.view(np.float32))
    assert np.array_equal(mine[~nan], ref[~nan])
    assert np.all((mine[nan] & 0x7C00) == 0x7C00) and np.all((mine[nan] & 0x03FF) != 0)


def _f16_row_perm(r):  # tile f row 4g+i <- feature 32(f>>1) + 8g + 4(f&1) + i
    f, rho = r >> 4, r & 15
    return 32 * (f >> 1) + 8 * (rho >> 2) + 4 * (f & 1) + (rho & 3)


def test_f16_row_permutation(outputs):
    perm = _f16_row_perm(np.arange(E))
    assert sorted(perm.tolist()) == list(range(E))
    w = np.arange(E * FH, dtype=np.float32).reshape(E, FH)
    assert np.array_equal(outputs("rows_f16.bin", np.float32).reshape(E, FH), w[perm])
    # a lane (g) of Y^T tiles 2k, 2k+1 holds the 8 consecutive features 32k + 8g .. +7 (one 16-B fp16 run)
    for k in range(E // 32):
        for g in range(4):
            feats = [_f16_row_perm(16 * (2 * k + t) + 4 * g + i) for t in range(2) for i in range(4)]
            assert feats == list(range(32 * k + 8 * g, 32 * k + 8 * g + 8))


def test_transpose_out(outputs):
    o = outputs("transpose_out.bin", np.float32).reshape(E, E)
    assert np.array_equal(o, np.arange(E * E, dtype=np.float32).reshape(E, E).T)


def _perm32(pos):  # 8g + j -> 4g + j (j < 4) | 16 + 4g + (j - 4)
    g, j = pos >> 3, pos & 7
    return np.where(j < 4, 4 * g + j, 16 + 4 * g + (j - 4))


def test_mlp_permutations(outputs):
    k = np.arange(E)
    perm1 = 32 * (k // 32) + 16 * ((k % 8) // 4) + 4 * ((k % 32) // 8) + (k % 4)
    w1 = np.arange(FH * E, dtype=np.float32).reshape(FH, E)
    assert np.array_equal(outputs("mlp1.bin", np.float32).reshape(FH, E), w1[:, perm1])
    assert sorted(perm1.tolist()) == list(range(E))
    c = np.arange(FH)
    perm2 = 32 * (c // 32) + _perm32(c % 32)
    w2 = np.arange(E * FH, dtype=np.float32).reshape(E, FH)
    assert np.array_equal(outputs("mlp2.bin", np.float32).reshape(E, FH), w2[:, perm2])


def test_feat_rows_images(outputs):
    o = outputs("feat_rows.bin", np.float32)
    assert o.size == (H * 96 + E) * ST
    qkv = np.arange(3 * H * 32 * E, dtype=np.float32).reshape(3, H, 32, E)
    wout = -np.arange(E * H * 32, dtype=np.float32).reshape(E, H * 32)
    scale = np.float32(1.4426950408889634) / np.sqrt(np.float32(32.0))
    ref = np.zeros(((H * 96 + E), ST), np.float32)
    r = np.arange(96)
    j, rr = r // 32, r % 32
    f, rho = rr >> 4, rr & 15
    dd = np.where(j < 2, 8 * (rho >> 2) + 4 * f + (rho & 3), rr)
    for h in range(H):
        rows = qkv[j, h, dd, :]
        rows = np.where((j == 0)[:, None], rows * scale, rows).astype(np.float32)
        ref[96 * h:96 * h + 96, :E] = rows
    cc = np.arange(H * 32)
    ref[H * 96:, :H * 32] = wout[:, 32 * (cc // 32) + _perm32(cc % 32)]
    assert np.array_equal(o.reshape(-1, ST), ref)


def test_feat_rows_images_f16(outputs):
    """PREC_F16 images: the QKV part as in bf16; the out-projection rows in f16_row_perm order."""
    o = outputs("feat_rows_f16.bin", np.float32).reshape(-1, ST)
    b = outputs("feat_rows.bin", np.float32).reshape(-1, ST)
    assert np.array_equal(o[:H * 96], b[:H * 96])
    assert np.array_equal(o[H * 96:], b[H * 96:][_f16_row_perm(np.arange(E))])


def test_fold_ln(outputs):
    n, k = np.meshgrid(np.arange(576), np.arange(E), indexing="ij")
    W = (((n * 7 + k * 3) % 17 - 8) / np.float32(8.0)).astype(np.float32)
    c = (np.arange(576) / np.float32(32.0)).astype(np.float32)
    g = (1.0 + np.arange(E) / np.float32(256.0)).astype(np.float32)
    b = (np.arange(E) / np.float32(1024.0) - np.float32(0.1)).astype(np.float32)
    Wf = outputs("fold_W.bin", np.float32).reshape(576, E)
    cf = outputs("fold_c.bin", np.float32)
    assert np.array_equal(Wf, (W * g).astype(np.float32))
    np.testing.assert_allclose(cf, c.astype(np.float64) + W.astype(np.float64) @ b.astype(np.float64), rtol=1e-6)


def test_siphash_rows(outputs):
    from multimodalpfn_amd.model._siphash import siphash24_rows_numpy

    got = outputs("siphash.bin", np.int64).reshape(-1, 5)
    for i, rb in enumerate([0, 1, 7, 8, 9, 15, 16, 17, 31, 33, 100, 768]):
        buf = ((np.arange(5 * rb + 1) * 31 + 7 + rb) & 255).astype(np.uint8)
        rows = buf[:5 * rb].reshape(5, rb)
        assert np.array_equal(got[i], np.asarray(siphash24_rows_numpy(rows), dtype=np.int64)), rb
