"""Analyse tools/probe/probe_mfma output (test infrastructure, not product code).

Checks (1) the int8 MFMA operand/accumulator lane maps used by the encoder kernels,
(2) that f32 MFMA chains equal a k-ordered fmaf chain, and (3) which accumulation model
reproduces bf16 MFMA bit-for-bit.
"""
import math
import sys

import numpy as np

D = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/probe"
NT = 512


def load(name, dt):
    return np.fromfile(f"{D}/{name}", dtype=dt)


def exact(v):
    """float -> (int mantissa, exponent) exactly."""
    if v == 0.0:
        return 0, 0
    m, e = math.frexp(float(v))
    return int(m * (1 << 53)), e - 53


def round_f32(S, E):
    """Round S*2^E (Python ints) to float32 with round-half-even."""
    if S == 0:
        return np.float32(0.0)
    sign = -1 if S < 0 else 1
    S = abs(S)
    nb = S.bit_length()
    # target: 24 significant bits, but not below exponent -149 (subnormal)
    exp_top = nb + E  # value in [2^(exp_top-1), 2^exp_top)
    lsb = max(exp_top - 24, -149)
    shift = lsb - E
    if shift > 0:
        q, r = divmod(S, 1 << shift)
        half = 1 << (shift - 1)
        if r > half or (r == half and (q & 1)):
            q += 1
        S, E = q, lsb
    return np.float32(sign * math.ldexp(float(S), E))


def exact_sum_round(terms):
    parts = [exact(t) for t in terms]
    parts = [p for p in parts if p[0] != 0]
    if not parts:
        return np.float32(0.0)
    emin = min(e for _, e in parts)
    S = sum(m << (e - emin) for m, e in parts)
    return round_f32(S, emin)


def check_i8():
    A = load("i8_A.bin", np.int8).reshape(NT, -1).astype(np.int64)
    B = load("i8_B.bin", np.int8).reshape(NT, -1).astype(np.int64)
    D16 = load("i8_D16.bin", np.int32).reshape(NT, 16, 16)
    D32 = load("i8_D32.bin", np.int32).reshape(NT, 32, 32)
    ref16 = np.einsum("tmk,tnk->tmn", A.reshape(NT, 16, 64), B.reshape(NT, 16, 64))
    ref32 = np.einsum("tmk,tnk->tmn", A.reshape(NT, 32, 32), B.reshape(NT, 32, 32))
    print("int8 16x16x64 layout ok:", np.array_equal(ref16, D16), " 32x32x32 ok:", np.array_equal(ref32, D32))


def check_f32():
    A = load("f32_A.bin", np.float32).reshape(NT, 16, 64)
    B = load("f32_B.bin", np.float32).reshape(NT, 16, 64)
    C = load("f32_C.bin", np.float32).reshape(NT, 16, 16)
    Dg = load("f32_D.bin", np.float32).reshape(NT, 16, 16)
    acc = C.astype(np.float32).copy()
    for k in range(64):
        p = A[:, :, k][:, :, None].astype(np.float64) * B[:, :, k][:, None, :].astype(np.float64)
        acc = (acc.astype(np.float64) + p).astype(np.float32)  # fmaf: exact product + one rounding
    # np float64 add of exact product and f32 acc then round: double rounding possible but rare
    eq = (acc.view(np.int32) == Dg.view(np.int32)).mean()
    print(f"f32 16x16x4 chained == fmaf chain: {eq*100:.4f}% bitwise")


def bf_models(a, b, c):
    """a,b: [K] float (bf16-valued) c: scalar. Return dict of model -> f32."""
    K = len(a)
    prods = [float(a[k]) * float(b[k]) for k in range(K)]  # exact in double
    out = {}
    acc = np.float32(c)
    for p in prods:
        acc = exact_sum_round([acc, p])
    out["seq_fma"] = acc
    out["exact_all"] = exact_sum_round(prods + [float(c)])
    s = exact_sum_round(prods)
    out["exact_then_c"] = exact_sum_round([s, float(c)])
    for G in (2, 4, 8, 16):
        if G >= K:
            continue
        acc = np.float32(c)
        for g in range(0, K, G):
            acc = exact_sum_round([acc] + prods[g:g + G])
        out[f"grpC_{G}"] = acc
        acc = np.float32(c)
        for g in range(0, K, G):
            acc = exact_sum_round([acc, exact_sum_round(prods[g:g + G])])
        out[f"grp_{G}"] = acc
    return out


def check_bf16(ntiles=24):
    for dist in range(5):
        A = load(f"bf_A{dist}.bin", np.uint16).reshape(NT, -1)
        B = load(f"bf_B{dist}.bin", np.uint16).reshape(NT, -1)
        C = load(f"bf_C{dist}.bin", np.float32).reshape(NT, -1)
        for shape in ("16", "32"):
            Dg = load(f"bf_D{shape}_{dist}.bin", np.float32)
            if shape == "16":
                M, K = 16, 32
                Dg = Dg.reshape(NT, 16, 16)
            else:
                M, K = 32, 16
                Dg = Dg.reshape(NT, 32, 32)
            Af = (A.astype(np.uint32) << 16).view(np.float32).reshape(NT, M, K)
            Bf = (B.astype(np.uint32) << 16).view(np.float32).reshape(NT, M, K)
            if shape == "16":
                Cf = C[:, :256].reshape(NT, 16, 16)
            else:
                Cf = C.reshape(NT, 32, 32)
            hits = {}
            total = 0
            for t in range(ntiles):
                for m in range(M):
                    for n in range(M):
                        res = bf_models(Af[t, m], Bf[t, n], Cf[t, m, n])
                        g = Dg[t, m, n]
                        total += 1
                        for k_, v in res.items():
                            hits[k_] = hits.get(k_, 0) + (np.float32(v).view(np.int32) == np.float32(g).view(np.int32))
            best = sorted(hits.items(), key=lambda kv: -kv[1])
            print(f"bf16 {shape}x{shape} dist{dist}: " + ", ".join(f"{k}={v/total*100:.2f}%" for k, v in best))


if __name__ == "__main__":
    check_i8()
    check_f32()
    check_bf16()
