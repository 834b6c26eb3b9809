"""CPU checks of the fast-convolution algebra the HIP kernels implement (numpy, fp64).

* The F(3x3,3x3), F(3x3,5x5) and F(4x4,5x5) tables in csrc/include/anx/winograd_f*.hpp (parsed from
  the headers the kernels compile against) reproduce direct correlation exactly in fp64.
* Conv2's tilings of its 31x31 window: 9x9 tiles of 3x3 outputs, and 7x7 tiles of 4x4 outputs whose
  last tile row / column reads window row / column 31 (outside the window: zero) for the output row
  27 that is dropped — the kernels' bounds logic (winograd.hip, wino_gemm16.hpp).
* Conv1's polyphase rewrite (stride 4 -> 48 channels of a stride-1 3x3 conv) followed by F(3x3,3x3)
  tiles equals the direct 11x11/4 convolution, including ragged right/bottom tiles — the exact data
  flow of hip/conv1_wino.hip (channel order ch = (rh*4 + rw)*3 + c, 12-pixel tile pitch).
"""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _table(text, name):
    m = re.search(r"%s\[(\d+)\]\[(\d+)\] = \{(.*?)\};" % name, text, re.S)
    rows, cols = int(m.group(1)), int(m.group(2))
    vals = [float(v.rstrip("f")) for v in re.findall(r"-?[0-9.]+(?:e-?\d+)?f?", m.group(3))]
    return np.array(vals, dtype=np.float64).reshape(rows, cols)


def _load(header):
    text = open(os.path.join(ROOT, "csrc/include/anx", header)).read()
    return _table(text, "kAT"), _table(text, "kBT"), _table(text, "kG")


def _wino2d(d, g, AT, BT, G):
    U = G @ g @ G.T
    V = BT @ d @ BT.T
    return AT @ (U * V) @ AT.T


@pytest.mark.parametrize("header,m,r", [("winograd_f33.hpp", 3, 3), ("winograd_f35.hpp", 3, 5),
                                        ("winograd_f45.hpp", 4, 5)])
def test_tables_exact(header, m, r):
    AT, BT, G = _load(header)
    n = m + r - 1
    assert AT.shape == (m, n) and BT.shape == (n, n) and G.shape == (n, r)
    rng = np.random.default_rng(0)
    for _ in range(20):
        d = rng.standard_normal((n, n))
        g = rng.standard_normal((r, r))
        ref = np.array([[(d[i:i + r, j:j + r] * g).sum() for j in range(m)] for i in range(m)])
        np.testing.assert_allclose(_wino2d(d, g, AT, BT, G), ref, rtol=1e-10, atol=1e-10)


def _conv1_direct(x, w, S=4):
    H, W, C = x.shape
    K, _, F, _ = w.shape
    Ho, Wo = (H - F) // S + 1, (W - F) // S + 1
    y = np.zeros((Ho, Wo, K))
    for oy in range(Ho):
        for ox in range(Wo):
            patch = x[oy * S:oy * S + F, ox * S:ox * S + F, :]  # F,F,C
            y[oy, ox] = np.einsum("hwc,kchw->k", patch, w)
    return y


def _conv1_polyphase_wino(x, w):
    """Mirror of conv1_wino_in_kernel + conv1_wino_weights_host + conv1_wino_gemm_kernel."""
    AT, BT, G = _load("winograd_f33.hpp")
    H, W, C = x.shape
    K, _, F, _ = w.shape
    H1, W1 = (H - F) // 4 + 1, (W - F) // 4 + 1
    ty, tx = (H1 + 2) // 3, (W1 + 2) // 3
    # U[a][b][k][ch], ch = (rh*4 + rw)*3 + c
    U = np.zeros((5, 5, K, 48))
    for ch in range(48):
        rh, rw, c = ch // 12, (ch % 12) // 3, ch % 3
        g = np.zeros((K, 3, 3))
        for qh in range(3):
            for qw in range(3):
                fh, fw = 4 * qh + rh, 4 * qw + rw
                if fh < F and fw < F:
                    g[:, qh, qw] = w[:, c, fh, fw]
        U[:, :, :, ch] = np.einsum("au,kuv,bv->abk", G, g, G)
    y = np.zeros((ty * 3, tx * 3, K))
    for ti in range(ty):
        for tj in range(tx):
            d = np.zeros((5, 5, 48))  # X' patch: image rows 12ti + 4u + rh, cols 12tj + 4v + rw
            for u in range(5):
                for v in range(5):
                    for ch in range(48):
                        rh, rw, c = ch // 12, (ch % 12) // 3, ch % 3
                        row, col = 12 * ti + 4 * u + rh, 12 * tj + 4 * v + rw
                        if row < H and col < W:
                            d[u, v, ch] = x[row, col, c]
            V = np.einsum("au,uvc,bv->abc", BT, d, BT)
            M = np.einsum("abc,abkc->abk", V, U)
            y[3 * ti:3 * ti + 3, 3 * tj:3 * tj + 3] = np.einsum("ia,abk,jb->ijk", AT, M, AT)
    return y[:H1, :W1]


@pytest.mark.parametrize("H,W", [(59, 47), (43, 63)])
def test_conv1_polyphase_winograd(H, W):
    rng = np.random.default_rng(1)
    x = rng.uniform(0, 0.1, (H, W, 3))
    w = rng.uniform(-0.01, 0.01, (8, 3, 11, 11))
    np.testing.assert_allclose(_conv1_polyphase_wino(x, w), _conv1_direct(x, w), rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("header,m", [("winograd_f35.hpp", 3), ("winograd_f45.hpp", 4)])
def test_conv2_window_tiling(header, m):
    AT, BT, G = _load(header)
    r, n, Hq, Ho = 5, m + 4, 31, 27
    rng = np.random.default_rng(1)
    C, K = 3, 2
    x = np.zeros((Hq, Hq, C))
    x[2:29, 2:29] = rng.standard_normal((27, 27, C))  # the zero border of the conv2 window
    w = rng.standard_normal((K, C, r, r))
    ty = -(-Ho // m)
    y = np.zeros((ty * m, ty * m, K))
    for ti in range(ty):
        for tj in range(ty):
            d = np.zeros((n, n, C))  # window rows / columns past 30 read as zero (the kernels' bounds checks)
            rr, cc = min(n, Hq - ti * m), min(n, Hq - tj * m)
            d[:rr, :cc] = x[ti * m:ti * m + rr, tj * m:tj * m + cc]
            for k in range(K):
                y[ti * m:(ti + 1) * m, tj * m:(tj + 1) * m, k] = sum(
                    _wino2d(d[:, :, c], w[k, c], AT, BT, G) for c in range(C))
    ref = np.zeros((Ho, Ho, K))
    for oy in range(Ho):
        for ox in range(Ho):
            ref[oy, ox] = np.einsum("hwc,kchw->k", x[oy:oy + r, ox:ox + r], w)
    np.testing.assert_allclose(y[:Ho, :Ho], ref, rtol=1e-9, atol=1e-9)
