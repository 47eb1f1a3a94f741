"""bf16 MFMA accumulation-model probe (test infrastructure, not product code).

    python tools/probe/probe_bf16.py gen DIR     # writes A.bin, Bt.bin, C.bin, cases.npz
    tools/probe/probe_bf16 DIR                   # on the GPU: D.bin
    python tools/probe/probe_bf16.py show DIR    # targeted-case tables
Each case is one output D[m][n] = C[m][n] + sum_k A[m][k] * Bt[n][k] of one
v_mfma_f32_16x16x32_bf16 (gfx950).
"""
import os
import sys
from fractions import Fraction

import numpy as np


def bf(x):
    """float64 -> bf16 bits (RNE) -- inputs here are chosen exactly representable."""
    f = np.asarray(x, np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def bf2f(b):
    return (np.asarray(b, np.uint32) << 16).view(np.float32)


class Gen:
    def __init__(self):
        self.A, self.B, self.C, self.meta = [], [], [], []
        self.cur = None

    def case(self, avec, cval, tag, bvec=None):
        """One targeted case: row m of A = avec (32 values), Bt rows = bvec (default ones)."""
        if self.cur is None or self.cur[3] == 16:
            self.cur = [np.zeros((16, 32), np.uint16), np.zeros((16, 32), np.uint16), np.zeros((16, 16), np.float32), 0]
            self.A.append(self.cur[0]); self.B.append(self.cur[1]); self.C.append(self.cur[2])
        m = self.cur[3]
        self.cur[0][m] = bf(avec)
        bvec = np.ones(32) if bvec is None else bvec
        self.cur[1][m] = bf(bvec)
        self.cur[2][m, m] = np.float32(cval)
        self.meta.append((len(self.A) - 1, m, m, tag))
        self.cur[3] += 1

    def tiles(self, A, B, C, tag):
        t0 = len(self.A)
        for i in range(A.shape[0]):
            self.A.append(A[i]); self.B.append(B[i]); self.C.append(C[i])
        self.cur = None
        return t0


def gen(d):
    os.makedirs(d, exist_ok=True)
    g = Gen()
    # E1: alignment of a small product against p0 = 1 at position p0
    for p0 in (0, 7, 8, 16, 31):
        for j in range(32):
            if j == p0:
                continue
            for s in range(1, 64):
                for sign in (1, -1):
                    a = np.zeros(32); a[p0] = 1.0; a[j] = sign * 2.0 ** -s
                    g.case(a, 0.0, f"E1 p0={p0} j={j} s={s} sign={sign}")
    # E2: C vs one product
    for s in range(-10, 64):
        for sign in (1, -1):
            a = np.zeros(32); a[5] = sign * 2.0 ** -s
            g.case(a, 1.0, f"E2a s={s} sign={sign}")
            a = np.zeros(32); a[5] = 1.0
            g.case(a, sign * 2.0 ** -s, f"E2b s={s} sign={sign}")
    # E3: sticky: 1 + 2^-24 (half ulp) + tiny
    for s in range(25, 64):
        for where in ("A", "C"):
            a = np.zeros(32); a[0] = 1.0; a[1] = 2.0 ** -24
            c = 0.0
            if where == "A":
                a[2] = 2.0 ** -s
            else:
                c = 2.0 ** -s
            g.case(a, c, f"E3 tiny_in={where} s={s}")
            a2 = a.copy(); a2[1] = -2.0 ** -24
            g.case(a2, c, f"E3neg tiny_in={where} s={s}")
    # E4: 1 + 31 small
    for s in range(18, 40):
        a = np.full(32, 2.0 ** -s); a[0] = 1.0
        g.case(a, 0.0, f"E4 s={s}")
        a = np.full(32, 2.0 ** -s); a[0] = 0.0
        g.case(a, 1.0, f"E4c s={s}")
    # E5: cancellation then small
    for big in (0, 4, 10, 30):
        for s in range(0, 64, 3):
            a = np.zeros(32); a[0] = 2.0 ** big; a[9] = -2.0 ** big; a[20] = 2.0 ** -s
            g.case(a, 0.0, f"E5 big={big} s={s}")
            a = np.zeros(32); a[0] = 2.0 ** big; a[20] = 2.0 ** -s
            g.case(a, -2.0 ** big, f"E5c big={big} s={s}")
    # E6: rounding direction for non-ties: 1 + 3*2^-25 (0.75 ulp) and negatives
    for frac in (1, 3, 5, 7):
        for sign in (1, -1):
            a = np.zeros(32); a[0] = sign * 1.0; a[3] = sign * frac * 2.0 ** -26
            g.case(a, 0.0, f"E6 frac={frac}/4ulp sign={sign}")
            a = np.zeros(32); a[3] = sign * frac * 2.0 ** -26
            g.case(a, sign * 1.0, f"E6c frac={frac}/4ulp sign={sign}")
    # E8: tie-breaking with a tiny extra term in the adder stage: C = 2^k (or its next float up),
    # products in group 1: half an ulp of C plus +-2^-s (relative to C's ulp)
    for k in (0, 5, -3):
        ulp = 2.0 ** (k - 23)
        for codd in (0, 1):
            c = 2.0 ** k + codd * ulp
            for csign in (1, -1):
                for s in range(1, 40):
                    for sign in (1, -1):
                        a = np.zeros(32); a[9] = csign * ulp / 2; a[12] = csign * sign * ulp * 2.0 ** -s
                        g.case(a, csign * c, f"E8 k={k} codd={codd} csign={csign} s={s} sign={sign}")
                        a = np.zeros(32); a[9] = csign * ulp / 2; a[20] = csign * sign * ulp * 2.0 ** -s
                        g.case(a, csign * c, f"E8x k={k} codd={codd} csign={csign} s={s} sign={sign}")
    # E7: random realistic tiles
    rng = np.random.default_rng(7)
    for dist in range(4):
        nt = 2048
        if dist == 0:  # weights x activations in (-1, 1), moderate C
            A = rng.normal(0, 0.05, (nt, 16, 32)); B = np.tanh(rng.normal(0, 1, (nt, 16, 32))); C = rng.normal(0, 0.5, (nt, 16, 16))
        elif dist == 1:  # wide exponent spread
            A = rng.normal(0, 1, (nt, 16, 32)) * 2.0 ** rng.integers(-12, 12, (nt, 16, 32))
            B = rng.normal(0, 1, (nt, 16, 32)) * 2.0 ** rng.integers(-12, 12, (nt, 16, 32))
            C = rng.normal(0, 1, (nt, 16, 16)) * 2.0 ** rng.integers(-12, 12, (nt, 16, 16))
        elif dist == 2:  # C = 0
            A = rng.normal(0, 1, (nt, 16, 32)); B = rng.normal(0, 1, (nt, 16, 32)); C = np.zeros((nt, 16, 16))
        else:  # large C, small products
            A = rng.normal(0, 0.01, (nt, 16, 32)); B = rng.normal(0, 1, (nt, 16, 32)); C = rng.normal(0, 30, (nt, 16, 16))
        g.tiles(bf(A), bf(B), C.astype(np.float32), f"E7 dist={dist}")
        g.meta.append((-1, dist, nt, f"E7 dist={dist} tiles"))
    A = np.stack(g.A); B = np.stack(g.B); C = np.stack(g.C)
    A.tofile(f"{d}/A.bin"); B.tofile(f"{d}/Bt.bin"); C.tofile(f"{d}/C.bin")
    np.save(f"{d}/meta.npy", np.array([str(m) for m in g.meta]))
    print("tiles", A.shape[0], "targeted cases", sum(1 for m in g.meta if m[0] >= 0))


def load(d):
    A = np.fromfile(f"{d}/A.bin", np.uint16).reshape(-1, 16, 32)
    B = np.fromfile(f"{d}/Bt.bin", np.uint16).reshape(-1, 16, 32)
    C = np.fromfile(f"{d}/C.bin", np.float32).reshape(-1, 16, 16)
    D = np.fromfile(f"{d}/D.bin", np.float32).reshape(-1, 16, 16)
    meta = [eval(m) for m in np.load(f"{d}/meta.npy")]
    return A, B, C, D, meta


def exact(t, m, n, A, B, C):
    a = bf2f(A[t, m]).astype(np.float64); b = bf2f(B[t, n]).astype(np.float64)
    return Fraction(float(C[t, m, n])) + sum(Fraction(float(x)) * Fraction(float(y)) for x, y in zip(a, b))


def show(d):
    A, B, C, D, meta = load(d)
    for t, m, n, tag in meta:
        if t < 0:
            continue
        ex = exact(t, m, n, A, B, C)
        got = Fraction(float(D[t, m, n]))
        rn = Fraction(float(np.float32(float(ex))))  # double then f32: near-RNE (fine for report)
        mark = "" if got == rn else "  <-- differs from round(exact)"
        if mark or tag.startswith(("E2", "E3", "E4", "E5", "E6")):
            print(f"{tag:40s} exact={float(ex):.10g} got={float(got):.10g} diff={float(got - ex):.3g}{mark}")


if __name__ == "__main__":
    {"gen": gen, "show": show}[sys.argv[1]](sys.argv[2])
