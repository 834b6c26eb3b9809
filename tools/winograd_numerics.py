import numpy as np
from fractions import Fraction as Fr
import itertools

def mats(m, r, pts):
    n = m + r - 1
    assert len(pts) == n - 1
    # Vandermonde n x n with infinity row
    V = [[Fr(p) ** j for j in range(n)] for p in pts] + [[Fr(0)] * (n - 1) + [Fr(1)]]
    Vm = [[Fr(p) ** j for j in range(m)] for p in pts] + [[Fr(0)] * (m - 1) + [Fr(1)]]
    Vr = [[Fr(p) ** j for j in range(r)] for p in pts] + [[Fr(0)] * (r - 1) + [Fr(1)]]
    import numpy.linalg as la
    Vf = np.array([[float(x) for x in row] for row in V])
    Vinv = la.inv(Vf)
    AT = np.array([[float(x) for x in row] for row in Vm]).T   # m x n
    G = np.array([[float(x) for x in row] for row in Vr])      # n x r
    BT = Vinv.T                                                # n x n
    # rescale: make each row of BT have integer-ish entries: scale row j of BT by s_j, G row j by 1/s_j
    for j in range(n):
        mx = np.max(np.abs(BT[j]))
        nz = np.abs(BT[j][np.abs(BT[j]) > 1e-12])
        s = 1.0 / nz.min()
        BT[j] *= s; G[j] /= s
    return AT, G, BT

def wino2d(d, g, AT, G, BT, dt=np.float32):
    # d: [C, n, n], g: [C, r, r] -> y [m, m]: sum over c
    U = np.einsum('ij,cjk,lk->cil', G.astype(dt), g.astype(dt), G.astype(dt))
    V = np.einsum('ij,cjk,lk->cil', BT.astype(dt), d.astype(dt), BT.astype(dt))
    M = (U * V).astype(dt).sum(0, dtype=dt)
    return (AT.astype(dt) @ M @ AT.T.astype(dt)).astype(dt)

def direct(d, g, m, r):
    y = np.zeros((m, m))
    for i in range(m):
        for j in range(m):
            y[i, j] = (d[:, i:i+r, j:j+r].astype(np.float64) * g.astype(np.float64)).sum()
    return y

rng = np.random.default_rng(0)
C = 96
for (m, pts) in [(2, [0, 1, -1, 2, -2]), (3, [0, 1, -1, 2, -2, 0.5]), (3, [0, 1, -1, 0.5, -0.5, 2]), (3,[0,1,-1,2,-2,-0.5])]:
    r = 5
    AT, G, BT = mats(m, r, pts)
    n = m + r - 1
    errs = []; rel = []
    for t in range(200):
        d = np.maximum(rng.normal(0.3, 1.0, (C, n, n)), 0).astype(np.float32)  # post-ReLU-ish
        g = (rng.uniform(-0.5, 0.5, (C, r, r)) * 0.02).astype(np.float32)
        y = wino2d(d, g, AT, G, BT)
        ref = direct(d, g, m, r)
        scale = direct(np.abs(d), np.abs(g), m, r)
        errs.append(np.abs(y - ref).max()); rel.append((np.abs(y - ref) / scale).max())
    # direct fp32 error for comparison
    e32 = []
    for t in range(50):
        d = np.maximum(rng.normal(0.3, 1.0, (C, n, n)), 0).astype(np.float32)
        g = (rng.uniform(-0.5, 0.5, (C, r, r)) * 0.02).astype(np.float32)
        y32 = np.zeros((m, m), np.float32)
        for i in range(m):
            for j in range(m):
                y32[i, j] = (d[:, i:i+r, j:j+r] * g).astype(np.float32).sum(dtype=np.float32)
        e32.append((np.abs(y32 - direct(d,g,m,r)) / direct(np.abs(d),np.abs(g),m,r)).max())
    print(f"F({m},{r}) pts={pts}: max abs err {max(errs):.3e}, max rel-to-|sum| {max(rel):.3e}; direct fp32 rel {max(e32):.3e}; max|BT|={np.abs(BT).max():.2f} max|G|={np.abs(G).max():.3f} max|AT|={np.abs(AT).max():.2f}")
