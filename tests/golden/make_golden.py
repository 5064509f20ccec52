"""Generate tests/golden/golden.npz — hand-derived known-answer vectors.

The reference ships no tests, fixtures or golden data, and its Pascal cannot
be compiled here, so nothing can be captured from a
reference run.  These vectors are instead derived *independently of the C
oracle*: a pure-Python transcription of the Pascal operation order using exact
rational arithmetic (fractions.Fraction) with one IEEE round-to-nearest-even
to binary32 per reference operation (an FMA is one rounding, a mul or add is
one rounding).  tests/test_oracle_golden.py then requires the C oracle to
reproduce every vector bit for bit.  Each case cites the Pascal it follows.

Run:  python tests/golden/make_golden.py   (deterministic; seeds below)
"""
from __future__ import annotations

import math
from fractions import Fraction
from pathlib import Path

import numpy as np

OUT = Path(__file__).resolve().parent / "golden.npz"


# ---------------------------------------------------------------- binary32
def f32(q) -> Fraction:
    """Round an exact rational to the nearest binary32 (ties to even)."""
    q = Fraction(q)
    if q == 0:
        return Fraction(0)
    sign = -1 if q < 0 else 1
    a = abs(q)
    e = math.floor(math.log2(a.numerator) - math.log2(a.denominator))
    # fix e so that 2^e <= a < 2^(e+1)
    while Fraction(2) ** e > a:
        e -= 1
    while Fraction(2) ** (e + 1) <= a:
        e += 1
    e = max(e, -126)                      # subnormal range keeps exponent -126
    scale = Fraction(2) ** (23 - e)       # 24-bit significand
    m = a * scale
    fl = m.numerator // m.denominator
    rem = m - fl
    if rem > Fraction(1, 2) or (rem == Fraction(1, 2) and fl % 2 == 1):
        fl += 1
    r = Fraction(fl) / scale
    if r >= Fraction(2) ** 128:
        raise OverflowError
    return sign * r


def F(x) -> Fraction:
    return Fraction(float(np.float32(x)))


def to_np(qs) -> np.ndarray:
    return np.array([float(q) for q in qs], dtype=np.float32)


def fma(a, b, c):
    return f32(a * b + c)


def add(a, b):
    return f32(a + b)


def mul(a, b):
    return f32(a * b)


# ---------------------------------------------------------------- kernels
def sdot(a, b):
    """sdot_avx2 SIMD_REGS=8 (ntensors.pas:1268-1303)."""
    n = len(a)
    acc = [Fraction(0)] * 8
    blocks = n // 8
    for t in range(blocks):
        for l in range(8):
            acc[l] = fma(a[8 * t + l], b[8 * t + l], acc[l])
    rem = n % 8
    if rem:
        for l in range(8):
            xa = a[8 * blocks + l] if l < rem else Fraction(0)
            xb = b[8 * blocks + l] if l < rem else Fraction(0)
            acc[l] = fma(xa, xb, acc[l])
    s = [add(acc[l], acc[l + 4]) for l in range(4)]
    return add(add(s[0], s[1]), add(s[2], s[3]))


def sgemm(ta, tb, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc):
    """cblas_sgemm (ntensors.pas:2231-2286) + s_nn/s_nt/s_tn/s_tt."""
    C = list(C)
    if beta != 1:
        for i in range(M):
            for j in range(N):
                C[i * ldc + j] = mul(beta, C[i * ldc + j])
    if not ta and not tb:        # s_nn 2061-2133: saxpy(N, ALPHA*A[kk], B_kk, C_i)
        for i in range(M):
            for kk in range(K):
                ap = mul(alpha, A[i * lda + kk])
                for j in range(N):
                    C[i * ldc + j] = fma(ap, B[kk * ldb + j], C[i * ldc + j])
    elif not ta and tb:          # s_nt 1957-1985
        for i in range(M):
            for j in range(N):
                s = mul(alpha, sdot(A[i * lda:i * lda + K], B[j * ldb:j * ldb + K]))
                C[i * ldc + j] = add(C[i * ldc + j], s)
    elif ta and not tb:          # s_tn 2007-2033
        for i in range(M):
            for kk in range(K):
                ap = mul(alpha, A[kk * lda + i])
                for j in range(N):
                    C[i * ldc + j] = fma(ap, B[kk * ldb + j], C[i * ldc + j])
    else:                        # s_tt 2159-2182: sum := sum + ALPHA*A*B (no FMA)
        for i in range(M):
            for j in range(N):
                s = Fraction(0)
                for kk in range(K):
                    s = add(s, mul(mul(alpha, A[i + kk * lda]), B[kk + j * ldb]))
                C[i * ldc + j] = add(C[i * ldc + j], s)
    return C


def out_dim(inp, pad, k, dil, stride):
    v = inp + 2 * pad - (dil * (k - 1) + 1)
    return int(v / stride) + 1


def im2col(C, H, W, kH, kW, pH, pW, sY, sX, dY, dX, im):
    """sim2Col (ntensors.pas:11415-11491)."""
    oh, ow = out_dim(H, pH, kH, dY, sY), out_dim(W, pW, kW, dX, sX)
    col = []
    for c in range(C):
        for kr in range(kH):
            for kc in range(kW):
                for orow in range(oh):
                    ir = -pH + kr * dY + orow * sY
                    for ocol in range(ow):
                        ic = -pW + kc * dX + ocol * sX
                        if 0 <= ir < H and 0 <= ic < W:
                            col.append(im[(c * H + ir) * W + ic])
                        else:
                            col.append(Fraction(0))
    return col


def col2im(C, H, W, kH, kW, pH, pW, sY, sX, dY, dX, col, im):
    """c2i / scol2im single-threaded order (ntensors.pas:11650-11763),
    including input_row := (kernel_row - pad) * dil."""
    oh, ow = out_dim(H, pH, kH, dY, sY), out_dim(W, pW, kW, dX, sX)
    im = list(im)
    ks = kH * kW
    for i in range(C * ks):
        chan, idx = divmod(i, ks)
        kr, kc = divmod(idx, kW)
        base = i * oh * ow
        for orow in range(oh):
            ir = (kr - pH) * dY + orow * sY
            if not (0 <= ir < H):
                continue
            for ocol in range(ow):
                ic = (kc - pW) * dX + ocol * sX
                if 0 <= ic < W:
                    p = (chan * H + ir) * W + ic
                    im[p] = add(im[p], col[base + orow * ow + ocol])
    return im


def leaky(x):
    """leaky_array (nactivation.pas:234-267): 0 > x ⇒ x*0.1f."""
    return [mul(F(0.1), v) if v < 0 else v for v in x]


def relu(x):
    """relu_activate (305-310): x*(x>0)."""
    return [mul(v, Fraction(1 if v > 0 else 0)) for v in x]


def add_bias(x, bias, F_, bs, batch):
    """vsAddB (ntensors.pas:4066-4093)."""
    x = list(x)
    for b in range(batch):
        for i in range(F_):
            for j in range(bs):
                p = (b * F_ + i) * bs + j
                x[p] = add(x[p], bias[i])
    return x


def vssum(a):
    """vssum_avx2 (ntensors.pas:3592-3620): 8 lanes over the full 8-blocks,
    lane_l + lane_{l+4}, haddps twice, then the remainder in order."""
    acc = [Fraction(0)] * 8
    nb = len(a) // 8
    for t in range(nb):
        for l in range(8):
            acc[l] = add(acc[l], a[8 * t + l])
    s = [add(acc[l], acc[l + 4]) for l in range(4)]
    r = add(add(s[0], s[1]), add(s[2], s[3]))
    for v in a[8 * nb:]:
        r = add(r, v)
    return r


def lanes_tail_fold(acc, tail_terms, quirk):
    """Common epilogue of srss (ntensors.pas:1508-1523) and sVarinceDelta_avx
    (8738-8756): with a tail, fold lanes l+4 into l and add the tail terms to
    lane 0; without one the fold is skipped (lanes 4..7 dropped) when quirk."""
    if not tail_terms and quirk:
        x = list(acc[:4])
    else:
        x = [add(acc[l], acc[l + 4]) for l in range(4)]
        for t in tail_terms:
            x[0] = add(x[0], t)
    return add(add(x[0], x[1]), add(x[2], x[3]))


def srss(mean, a, quirk):
    """srss (ntensors.pas:1493-1523): lanes of (mean - a)^2."""
    acc = [Fraction(0)] * 8
    nb = len(a) // 8
    for t in range(nb):
        for l in range(8):
            d = f32(mean - a[8 * t + l])
            acc[l] = add(acc[l], mul(d, d))
    tail = []
    for v in a[8 * nb:]:
        d = f32(mean - v)
        tail.append(mul(d, d))
    return lanes_tail_fold(acc, tail, quirk)


def var_delta_avx(mean, delta, x, quirk):
    """sVarinceDelta_avx (ntensors.pas:8721-8757): lanes of (x - mean)*delta."""
    acc = [Fraction(0)] * 8
    nb = len(x) // 8
    for t in range(nb):
        for l in range(8):
            k = 8 * t + l
            acc[l] = add(acc[l], mul(f32(x[k] - mean), delta[k]))
    tail = [mul(f32(x[k] - mean), delta[k]) for k in range(8 * nb, len(x))]
    return lanes_tail_fold(acc, tail, quirk)


def mean_var_delta_sums(delta, x, mean, groups, N, bs, quirk):
    """sMeanAndVarianceDelta (ntensors.pas:8831-8871) before the final
    scaling: per channel m = sum_j vsSumI(block), v = sum_j
    sVarinceDelta_avx(block), groups in order."""
    ms, vs = [], []
    for i in range(N):
        m = v = Fraction(0)
        for j in range(groups):
            o = (i + j * N) * bs
            m = add(m, vssum(delta[o:o + bs]))
            v = add(v, var_delta_avx(mean[i], delta[o:o + bs], x[o:o + bs], quirk))
        ms.append(m)
        vs.append(v)
    return ms, vs


def means_and_vars(x, groups, N, bs, quirk):
    """MeansAndVars (ntensors.pas:9102-9177) with vssum_avx2 / srss blocks."""
    S, S2 = F(groups * bs), F(groups * bs - 1)
    ms, vs = [], []
    for i in range(N):
        m = Fraction(0)
        for j in range(groups):
            o = (i + j * N) * bs
            m = add(m, vssum(x[o:o + bs]))
        m = f32(m / S)
        v = Fraction(0)
        for j in range(groups):
            o = (i + j * N) * bs
            v = add(v, srss(m, x[o:o + bs], quirk))
        ms.append(m)
        vs.append(f32(v / S2))
    return ms, vs


# ---------------------------------------------------------------- cases
def rnd(rng, n, lo=-1.0, hi=1.0):
    v = rng.uniform(lo, hi, n).astype(np.float32)
    return v, [F(t) for t in v]


def main() -> None:
    rng = np.random.default_rng(20250808)
    g: dict[str, np.ndarray] = {}

    # sdot lane order: cancellation-heavy vector where lane order matters
    for n in (13, 8, 5, 37):
        a, aq = rnd(rng, n, -1e3, 1e3)
        b, bq = rnd(rng, n)
        g[f"sdot_{n}_a"], g[f"sdot_{n}_b"] = a, b
        g[f"sdot_{n}_out"] = to_np([sdot(aq, bq)])

    gemm_cases = [
        # name, ta, tb, M, N, K, alpha, beta
        ("nn_a1b0", 0, 0, 5, 7, 13, 1.0, 0.0),
        ("nn_a05b2", 0, 0, 6, 9, 11, 0.5, 2.0),
        ("nn_a1b1", 0, 0, 4, 33, 17, 1.0, 1.0),
        ("nt_a1b0", 0, 1, 5, 6, 19, 1.0, 0.0),
        ("nt_a05b2", 0, 1, 3, 4, 8, 0.5, 2.0),
        ("tn_a1b0", 1, 0, 7, 5, 9, 1.0, 0.0),
        ("tn_a2b05", 1, 0, 4, 6, 10, 2.0, 0.5),
        ("tt_a1b0", 1, 1, 5, 4, 12, 1.0, 0.0),
        ("tt_a05b1", 1, 1, 3, 5, 7, 0.5, 1.0),
    ]
    for name, ta, tb, M, N, K, al, be in gemm_cases:
        lda = M if ta else K
        ldb = K if tb else N
        A, Aq = rnd(rng, (K if ta else M) * lda)
        B, Bq = rnd(rng, (N if tb else K) * ldb)
        Cm, Cq = rnd(rng, M * N)
        out = sgemm(ta, tb, M, N, K, F(al), Aq, lda, Bq, ldb, F(be), Cq, N)
        g[f"gemm_{name}_A"], g[f"gemm_{name}_B"], g[f"gemm_{name}_C"] = A, B, Cm
        g[f"gemm_{name}_dims"] = np.array([ta, tb, M, N, K, lda, ldb], np.int64)
        g[f"gemm_{name}_ab"] = np.array([al, be], np.float32)
        g[f"gemm_{name}_out"] = to_np(out)

    # beta = 0 is 0*C: NaN / Inf in C propagate (ntensors.pas:2259-2261)
    A, Aq = rnd(rng, 2 * 3)
    B, Bq = rnd(rng, 3 * 2)
    Cm = np.array([np.nan, 1.0, np.inf, -2.0], np.float32)
    g["beta0nan_A"], g["beta0nan_B"], g["beta0nan_C"] = A, B, Cm
    # expected: NaN, finite, NaN (0*inf), finite
    fin = sgemm(0, 0, 2, 2, 3, Fraction(1), Aq, 3, Bq, 2, Fraction(0),
                [Fraction(0)] * 4, 2)
    exp = to_np(fin)
    exp[0] = np.nan
    exp[2] = np.nan
    g["beta0nan_out"] = exp

    # im2col / col2im geometries: (C,H,W,k,pad,stride,dil)
    geos = [(2, 5, 4, 3, 1, 2, 2), (3, 6, 6, 3, 1, 1, 1), (1, 7, 5, 1, 0, 2, 1),
            (2, 4, 5, 3, 0, 1, 1), (1, 6, 6, 3, 2, 2, 2)]
    for gi, (C, H, W, k, p, s, d) in enumerate(geos):
        im, imq = rnd(rng, C * H * W)
        col = im2col(C, H, W, k, k, p, p, s, s, d, d, imq)
        g[f"i2c_{gi}_geo"] = np.array([C, H, W, k, p, s, d], np.int64)
        g[f"i2c_{gi}_im"] = im
        g[f"i2c_{gi}_col"] = to_np(col)
        colin, colq = rnd(rng, len(col))
        base, baseq = rnd(rng, C * H * W)
        g[f"c2i_{gi}_colin"] = colin
        g[f"c2i_{gi}_base"] = base
        g[f"c2i_{gi}_out"] = to_np(col2im(C, H, W, k, k, p, p, s, s, d, d, colq, baseq))

    # bias + leaky / relu
    x, xq = rnd(rng, 2 * 3 * 5)
    bias, bq = rnd(rng, 3)
    yb = add_bias(xq, bq, 3, 5, 2)
    g["bias_x"], g["bias_b"] = x, bias
    g["bias_out"] = to_np(yb)
    g["leaky_out"] = to_np(leaky(yb))
    g["relu_out"] = to_np(relu(yb))

    # batch-norm block reductions: vssum / srss / sVarinceDelta_avx lane
    # orders, tail and tail-less blocks, both settings of the quirk
    for n in (5, 8, 13, 16, 37, 64, 67):
        a, aq = rnd(rng, n, -2.0, 3.0)
        d, dq = rnd(rng, n)
        mu, muq = rnd(rng, 1, -0.5, 0.5)
        g[f"bn_{n}_a"], g[f"bn_{n}_d"], g[f"bn_{n}_mu"] = a, d, mu
        g[f"bn_{n}_vssum"] = to_np([vssum(aq)])
        for q in (0, 1):
            g[f"bn_{n}_srss_q{q}"] = to_np([srss(muq[0], aq, q)])
            g[f"bn_{n}_vdelta_q{q}"] = to_np([var_delta_avx(muq[0], dq, aq, q)])
    for gi, (groups, N, bs) in enumerate([(3, 2, 16), (2, 3, 13), (4, 1, 9)]):
        n = groups * N * bs
        x, xq = rnd(rng, n, -2.0, 2.0)
        d, dq = rnd(rng, n)
        g[f"bnc_{gi}_dims"] = np.array([groups, N, bs], np.int64)
        g[f"bnc_{gi}_x"], g[f"bnc_{gi}_d"] = x, d
        for q in (0, 1):
            m, v = means_and_vars(xq, groups, N, bs, q)
            g[f"bnc_{gi}_mean_q{q}"], g[f"bnc_{gi}_var_q{q}"] = to_np(m), to_np(v)
            ms, vs = mean_var_delta_sums(dq, xq, m, groups, N, bs, q)
            g[f"bnc_{gi}_msum_q{q}"], g[f"bnc_{gi}_vsum_q{q}"] = to_np(ms), to_np(vs)

    np.savez_compressed(OUT, **g)
    print(f"wrote {OUT} ({len(g)} arrays)")


if __name__ == "__main__":
    main()
