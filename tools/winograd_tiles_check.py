#!/usr/bin/env python3
"""fp32 error of every Winograd point set the kernels use, from the generated headers themselves.

For each csrc/include/anx/winograd_f*.hpp: random post-ReLU-like inputs and small weights over C
channels, one output tile computed the way the kernels do (U = G g G^T rounded once from fp64, V =
B^T d B and the product / sum / output transform in fp32), compared with the fp64 direct sum; the
printed number is max |error| / sum |x*w| over 100 tiles (profiles/r03_f4_numerics.txt).

usage: tools/winograd_tiles_check.py
"""
import os
import re

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(fn):
    s = open(fn).read()

    def mat(name, dt):
        m = re.search(name + r"\[(\d+)\]\[(\d+)\] = \{(.*?)\};", s, re.S)
        r, c = int(m.group(1)), int(m.group(2))
        vals = [float(x.rstrip("f")) for x in re.findall(r"-?[\d.]+(?:e-?\d+)?f?", m.group(3))]
        return np.array(vals, dtype=dt).reshape(r, c)

    return mat("kAT", np.float32), mat("kBT", np.float32), mat("kG", np.float64)


def main():
    rng = np.random.default_rng(1)
    for name, C in [("winograd_f45.hpp", 96), ("winograd_f43.hpp", 48), ("winograd_f35.hpp", 96),
                    ("winograd_f33.hpp", 48)]:
        fn = os.path.join(ROOT, "csrc", "include", "anx", name)
        AT, BT, G = load(fn)
        m, n = AT.shape
        r = G.shape[1]
        worst = 0.0
        for _ in range(100):
            d = np.maximum(rng.normal(0.3, 1, (C, n, n)), 0).astype(np.float32)
            g = (rng.uniform(-0.5, 0.5, (C, r, r)) * 0.02).astype(np.float32)
            U = np.einsum("ij,cjk,lk->cil", G, g.astype(np.float64), G).astype(np.float32)
            V = np.einsum("ij,cjk,lk->cil", BT, d, BT, dtype=np.float32)
            M = (U * V).sum(0, dtype=np.float32)
            y = (AT @ M @ AT.T).astype(np.float32)
            ref, sc = np.zeros((m, m)), np.zeros((m, m))
            for i in range(m):
                for j in range(m):
                    ref[i, j] = (d[:, i:i + r, j:j + r].astype(np.float64) * g).sum()
                    sc[i, j] = (np.abs(d[:, i:i + r, j:j + r]).astype(np.float64) * np.abs(g)).sum()
            worst = max(worst, (np.abs(y - ref) / sc).max())
        print(f"csrc/include/anx/{name} {worst}")


if __name__ == "__main__":
    main()
