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


# ---------------------------------------------------------------- round 3:
# batch-norm elementwise passes, softmax / cross-entropy, transcendental
# activations, the SGD update and one whole connected-layer train step.
# Decisions shared with the C oracle (stated there too): sEPSILON
# (ntensors.pas:95) is the single 1e-6; FPC's exp / ln / Power return
# extended, transcribed here as the C library's double exp / log / pow
# rounded once to single (math.exp/log/pow are the same libm calls).
EPS = F(1e-6)


def fsqrt(v):
    """sqrt of a binary32 rounded to binary32: the double sqrt is correctly
    rounded and 53 >= 2*24 + 2, so rounding it again to 24 bits is exact."""
    return f32(Fraction(math.sqrt(float(v))))


def fdiv(a, b):
    return f32(a / b)


def fsub(a, b):
    return f32(a - b)


def fexp(x):
    """exp of a single, FPC extended result assigned to a single (+inf when
    it overflows single)."""
    try:
        return f32(Fraction(math.exp(float(x))))
    except OverflowError:
        return math.inf


def fmax(a, b):
    return a if a > b else b


def block_normalize(x, groups, N, bs, means, var):
    """TTensor.blockNormalize (ntensors.pas:8693-8718): blockSize 1 ->
    normvv = _snormvv (4331-4342): (x - m) / sqrt(max(v, eps)); otherwise
    normblkvv = _snormblkvv (4357-4382) -> snormvss: d := max(sqrt(v), eps),
    (x - m) / d (the AVX form snormvss_avx uses rcpss: quirk 5, not used)."""
    x = list(x)
    for g in range(groups):
        for i in range(N):
            o = (g * N + i) * bs
            if bs == 1:
                x[o] = fdiv(fsub(x[o], means[i]), fsqrt(fmax(var[i], EPS)))
            else:
                d = fmax(fsqrt(var[i]), EPS)
                for j in range(bs):
                    x[o + j] = fdiv(fsub(x[o + j], means[i]), d)
    return x


def forward_scale(x, groups, N, bs, s):
    """TTensor.forwardScale (7687-7707) -> mulblkvv / vsMulB (4112-4139):
    c[j] := c[j] * s[i], one rounding."""
    x = list(x)
    for g in range(groups):
        for i in range(N):
            o = (g * N + i) * bs
            for j in range(bs):
                x[o + j] = mul(x[o + j], s[i])
    return x


def normalize_delta(x, means, var, md, vd, delta, groups, N, bs):
    """sNormalizeDelta (8902-8951) with sNormalizeDelta_avx (8761-8818):
    arguments md/B, 2*vd/B, mean, sqrt(max(v, eps)) (8935, B = groups*bs);
    per element a := d / std; t := (x - mean) * vdB; t := t + mdB;
    d := a + t (vdivps, vsubps, vmulps, vaddps, vaddps: each rounded)."""
    delta = list(delta)
    B = F(groups * bs)
    for j in range(groups):
        for i in range(N):
            mdb = fdiv(md[i], B)
            vdb = fdiv(mul(F(2), vd[i]), B)
            sd = fsqrt(fmax(var[i], EPS))
            o = (i + j * N) * bs
            for k in range(bs):
                a = fdiv(delta[o + k], sd)
                t = add(mul(fsub(x[o + k], means[i]), vdb), mdb)
                delta[o + k] = add(a, t)
    return delta


def strided_sum(vals):
    """vsSumI with stride != 1 (3624-3635): Result := Result + src[i]."""
    r = Fraction(0)
    for v in vals:
        r = add(r, v)
    return r


def add_sums(dst, src, groups, N, bs):
    """TTensor.addSums (7729-7781): blockSize 1 -> sumv(groups, D2+i, nDst),
    which is vssum_avx2 when the stride nDst is 1 and the scalar loop
    otherwise; else per channel the group blocks' vssum in group order."""
    dst = list(dst)
    for i in range(N):
        if bs == 1:
            vals = [src[g * N + i] for g in range(groups)]
            dst[i] = add(dst[i], vssum(vals) if N == 1 else strided_sum(vals))
        else:
            s = Fraction(0)
            for g in range(groups):
                o = (g * N + i) * bs
                s = add(s, vssum(src[o:o + bs]))
            dst[i] = add(dst[i], s)
    return dst


def add_dots(dst, a, b, groups, N, bs):
    """TTensor.addDots (7783-7834): blockSize 1 -> dotvv(groups, stride
    nDst) = cblas_sdot's strided loop (2217-2219: mul, then add); else per
    group block sdot (8-lane FMA) summed in group order."""
    dst = list(dst)
    for i in range(N):
        if bs == 1:
            r = Fraction(0)
            for g in range(groups):
                r = add(r, mul(a[g * N + i], b[g * N + i]))
            dst[i] = add(dst[i], r)
        else:
            s = Fraction(0)
            for g in range(groups):
                o = (i + g * N) * bs
                s = add(s, sdot(a[o:o + bs], b[o:o + bs]))
            dst[i] = add(dst[i], s)
    return dst


def mean_var_delta(delta, x, means, var, groups, N, bs, quirk):
    """sMeanAndVarianceDelta (8831-8871), final scaling included:
    mean_delta = m * (-1 / sqrt(max(v, eps))) in single;
    variance_delta = v * -0.5 * Power(max(v, eps), -1.5) in double."""
    ms, vs = mean_var_delta_sums(delta, x, means, groups, N, bs, quirk)
    md, vd = [], []
    for i in range(N):
        ve = fmax(var[i], EPS)
        md.append(mul(ms[i], fdiv(F(-1), fsqrt(ve))))
        vd.append(f32(Fraction(float(vs[i]) * -0.5 * math.pow(float(ve), -1.5))))
    return md, vd


def logistic(x):
    """logistic_activate (nactivation.pas:293-297): 1/(1 + exp(-x)) in the
    extended evaluation (here double), rounded once."""
    return [f32(Fraction(1.0 / (1.0 + math.exp(-float(v))))) for v in x]


def tanh_act(x):
    """tanh_activate (351-360): px := exp(x); nx := exp(-x) as singles,
    (px - nx)/(px + nx) in single."""
    out = []
    for v in x:
        px, nx = fexp(v), fexp(-v)
        if math.inf in (px, nx):   # inf - x over inf + x: NaN (IEEE, exact)
            out.append(math.nan)
            continue
        out.append(fdiv(fsub(px, nx), add(px, nx)))
    return out


def activate(x, act):
    if act == 0:
        return logistic(x)
    if act == 1:
        return relu(x)
    if act == 4:
        return list(x)
    if act == 6:
        return tanh_act(x)
    if act == 9:
        return leaky(x)
    raise ValueError(act)


def gradient(y, act, delta):
    """gradient_array (nactivation.pas:624-717): delta *= f'(y) with
    logistic (1 - y)*y (423-426), relu ord(y > 0), linear 1, tanh 1 - y*y,
    leaky y > 0 ? 1 : 0.1."""
    out = []
    for v, d in zip(y, delta):
        if act == 0:
            g = mul(fsub(F(1), v), v)
        elif act == 1:
            g = Fraction(1 if v > 0 else 0)
        elif act == 4:
            out.append(d)
            continue
        elif act == 6:
            g = fsub(F(1), mul(v, v))
        elif act == 9:
            g = Fraction(1) if v > 0 else F(0.1)
        else:
            raise ValueError(act)
        out.append(mul(d, g))
    return out


def softmax(xs, temp):
    """softmax (nsoftmaxlayer.pas:83-106): largest, e := exp((x - largest) /
    temp) as a single, sum := sum + e, then o := o / sum."""
    largest = xs[0]
    for v in xs[1:]:
        if v > largest:
            largest = v
    es, s = [], Fraction(0)
    for v in xs:
        e = fexp(fdiv(fsub(v, largest), temp))
        s = add(s, e)
        es.append(e)
    return [fdiv(e, s) for e in es]


def softmax_xent(pred, truth):
    """softmaxCrossEntropy (123-137): error := -ln(max(p, eps)) where t <> 0,
    else 0; delta := t - p."""
    err, dl = [], []
    for p, t in zip(pred, truth):
        err.append(f32(Fraction(-math.log(float(fmax(p, EPS))))) if t != 0 else Fraction(0))
        dl.append(fsub(t, p))
    return dl, err


def sgd_update(W, dW, b, db, scales, dscales, lr, momentum, decay, batch):
    """TConnectedLayer.update (nconnectedlayer.pas:324-359): lrb :=
    learningRate / batch, ndb := -decay * batch (singles);
    biases.axpy(lrb, bias_updates) (saxpy: FMA); bias_updates *= momentum;
    scales likewise; weight_updates.axpy(ndb, weights);
    weights.axpy(lrb, weight_updates); weight_updates *= momentum."""
    lrb = fdiv(lr, F(batch))
    ndb = mul(-decay, F(batch))
    b = [fma(lrb, g, v) for v, g in zip(b, db)]
    db = [mul(momentum, g) for g in db]
    if scales is not None:
        scales = [fma(lrb, g, v) for v, g in zip(scales, dscales)]
        dscales = [mul(momentum, g) for g in dscales]
    dW = [fma(ndb, w, g) for w, g in zip(W, dW)]
    W = [fma(lrb, g, w) for w, g in zip(W, dW)]
    dW = [mul(momentum, g) for g in dW]
    return W, dW, b, db, scales, dscales


def mlp_step(widths, acts, B, X, T, layers, lr, momentum, decay):
    """One TNNet train step over connected layers with batch norm and a
    softmax layer (nnet.pas:275-450): per layer forward (nconnectedlayer.pas
    157-242): out := X . W^T (gemm NT: sdot per element), MeansAndVars
    (blockSize 1), rolling stats Multiply(1 - 0.05) then axpy(0.05, stat),
    x := out, blockNormalize, x_norm := out, forwardScale, forwardBias,
    activate; softmax + cross-entropy, cost = loss.Sum() (vssum_avx2);
    backward (244-322): the softmax delta added into the last layer's delta
    (zeroed in forward), Clamp(-1, 1), gradient, addSums, addDots,
    forwardScale, MeansAndVarsDelta, normalizeDelta, dW += delta^T . X (TN,
    beta 1), prev delta += delta . W (NN, beta 1; none for layer 0); then
    update every layer.  `layers` holds each layer's dict of lists."""
    mom = F(0.05)
    keep = fsub(F(1), mom)
    inp = X
    for li, L in enumerate(layers):
        I, O = widths[li], widths[li + 1]
        L["delta"] = [Fraction(0)] * (B * O)
        out = sgemm(0, 1, B, O, I, Fraction(1), inp, I, L["W"], I, Fraction(0),
                    [Fraction(0)] * (B * O), O)
        m, v = means_and_vars(out, B, O, 1, 0)
        L["mean"], L["var"] = m, v
        L["rmean"] = [fma(mom, s, mul(r, keep)) for r, s in zip(L["rmean"], m)]
        L["rvar"] = [fma(mom, s, mul(r, keep)) for r, s in zip(L["rvar"], v)]
        L["x"] = list(out)
        out = block_normalize(out, B, O, 1, m, v)
        L["xnorm"] = list(out)
        out = forward_scale(out, B, O, 1, L["scales"])
        out = add_bias(out, L["b"], O, 1, B)
        L["out"] = activate(out, acts[li])
        inp = L["out"]
    C = widths[-1]
    sm = []
    for r in range(B):
        sm += softmax(inp[r * C:(r + 1) * C], Fraction(1))
    sm_delta, loss = softmax_xent(sm, T)
    cost = vssum(loss)
    last = layers[-1]
    last["delta"] = [add(d, s) for d, s in zip(last["delta"], sm_delta)]
    for li in range(len(layers) - 1, -1, -1):
        L = layers[li]
        I, O = widths[li], widths[li + 1]
        lin = X if li == 0 else layers[li - 1]["out"]
        d = [fmax(F(-1), v) if v < -1 else (F(1) if v > 1 else v) for v in L["delta"]]
        d = gradient(L["out"], acts[li], d)
        L["db"] = add_sums(L["db"], d, B, O, 1)
        L["dscales"] = add_dots(L["dscales"], L["xnorm"], d, B, O, 1)
        d = forward_scale(d, B, O, 1, L["scales"])
        md, vd = mean_var_delta(d, L["x"], L["mean"], L["var"], B, O, 1, 0)
        L["mdelta"], L["vdelta"] = md, vd
        d = normalize_delta(L["x"], L["mean"], L["var"], md, vd, d, B, O, 1)
        L["delta"] = d
        L["dW"] = sgemm(1, 0, O, I, B, Fraction(1), d, O, lin, I, Fraction(1), L["dW"], I)
        if li > 0:
            P = layers[li - 1]
            P["delta"] = sgemm(0, 0, B, I, O, Fraction(1), d, O, L["W"], I, Fraction(1),
                               P["delta"], I)
    for L in layers:
        (L["W"], L["dW"], L["b"], L["db"], L["scales"],
         L["dscales"]) = sgd_update(L["W"], L["dW"], L["b"], L["db"], L["scales"],
                                    L["dscales"], lr, momentum, decay, B)
    return cost, sm, sm_delta, loss


MLP_ORDER = ["W", "b", "dW", "db", "scales", "rmean", "rvar", "dscales", "out", "delta", "x",
             "xnorm", "mean", "var", "mdelta", "vdelta"]


def mlp_sizes(I, O, B):
    return {"W": I * O, "b": O, "dW": I * O, "db": O, "scales": O, "rmean": O, "rvar": O,
            "dscales": O, "out": B * O, "delta": B * O, "x": B * O, "xnorm": B * O, "mean": O,
            "var": O, "mdelta": O, "vdelta": O}


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

    # ---- round 3 cases
    # blockNormalize, both epsilon forms; forwardScale; sNormalizeDelta
    for gi, (groups, N, bs) in enumerate([(4, 3, 1), (3, 2, 16), (2, 3, 13), (5, 1, 1)]):
        n = groups * N * bs
        x, xq = rnd(rng, n, -2.0, 2.0)
        d, dq = rnd(rng, n)
        sc, scq = rnd(rng, N, 0.5, 1.5)
        m, v = means_and_vars(xq, groups, N, bs, 0)
        if gi == 0:     # one channel with a variance under eps: the max() matters
            v[1] = F(3e-7)
        mq, mqs = to_np(m), m
        g[f"bnn_{gi}_dims"] = np.array([groups, N, bs], np.int64)
        g[f"bnn_{gi}_x"], g[f"bnn_{gi}_d"], g[f"bnn_{gi}_s"] = x, d, sc
        g[f"bnn_{gi}_mean"], g[f"bnn_{gi}_var"] = mq, to_np(v)
        g[f"bnn_{gi}_norm"] = to_np(block_normalize(xq, groups, N, bs, mqs, v))
        g[f"bnn_{gi}_scaled"] = to_np(forward_scale(xq, groups, N, bs, scq))
        md, vd = mean_var_delta(dq, xq, mqs, v, groups, N, bs, 0)
        g[f"bnn_{gi}_md"], g[f"bnn_{gi}_vd"] = to_np(md), to_np(vd)
        g[f"bnn_{gi}_ndelta"] = to_np(normalize_delta(xq, mqs, v, md, vd, dq, groups, N, bs))
        acc, accq = rnd(rng, N)
        g[f"bnn_{gi}_acc"] = acc
        g[f"bnn_{gi}_dots"] = to_np(add_dots(accq, xq, dq, groups, N, bs))
        g[f"bnn_{gi}_sums"] = to_np(add_sums(accq, dq, groups, N, bs))

    # logistic / tanh (incl. large |x| where exp overflows single -> NaN tanh)
    xa = np.concatenate([rng.uniform(-8, 8, 40), [0.0, -0.0, 30.0, -30.0, 88.0, 89.0, -89.0,
                                                   1e-8, -17.5]]).astype(np.float32)
    xaq = [F(t) for t in xa]
    g["act_x"] = xa
    g["act_logistic"] = to_np(logistic(xaq))
    g["act_tanh"] = to_np(tanh_act(xaq))
    dg, dgq = rnd(rng, len(xa))
    ya = to_np(logistic(xaq))
    g["grad_d"] = dg
    g["grad_logistic"] = to_np(gradient([F(t) for t in ya], 0, dgq))
    yt = np.tanh(xa.astype(np.float64)).astype(np.float32)
    g["grad_tanh_y"] = yt
    g["grad_tanh"] = to_np(gradient([F(t) for t in yt], 6, dgq))

    # softmax rows (temperature 1 and 0.5) + cross-entropy with one-hot truth
    for gi, (rows, n, temp) in enumerate([(3, 10, 1.0), (2, 7, 0.5)]):
        xs, xsq = rnd(rng, rows * n, -6.0, 6.0)
        sm = []
        for r in range(rows):
            sm += softmax(xsq[r * n:(r + 1) * n], F(temp))
        tr = np.zeros(rows * n, np.float32)
        tr[[r * n + (r * 3) % n for r in range(rows)]] = 1.0
        dl, err = softmax_xent(sm, [F(t) for t in tr])
        g[f"sm_{gi}_dims"] = np.array([rows, n], np.int64)
        g[f"sm_{gi}_temp"] = np.array([temp], np.float32)
        g[f"sm_{gi}_x"], g[f"sm_{gi}_truth"] = xs, tr
        g[f"sm_{gi}_out"], g[f"sm_{gi}_delta"] = to_np(sm), to_np(dl)
        g[f"sm_{gi}_err"] = to_np(err)
        g[f"sm_{gi}_cost"] = to_np([vssum(err)])

    # connected-layer SGD update (with and without scales)
    nw, no = 23, 5
    W, Wq = rnd(rng, nw)
    dW, dWq = rnd(rng, nw, -0.1, 0.1)
    b, bq = rnd(rng, no)
    db, dbq = rnd(rng, no)
    s_, sq_ = rnd(rng, no, 0.5, 1.5)
    ds, dsq = rnd(rng, no)
    hyper = np.array([0.01, 0.9, 0.0005], np.float32)
    hq = [F(t) for t in hyper]
    g["sgd_W"], g["sgd_dW"], g["sgd_b"], g["sgd_db"] = W, dW, b, db
    g["sgd_s"], g["sgd_ds"], g["sgd_hyper"] = s_, ds, hyper
    g["sgd_batch"] = np.array([32], np.int64)
    for tag, useS in (("bn", True), ("nobn", False)):
        res = sgd_update(Wq, dWq, bq, dbq, sq_ if useS else None, dsq if useS else None,
                         hq[0], hq[1], hq[2], 32)
        for k, arr in zip(("W", "dW", "b", "db", "s", "ds"), res):
            if arr is not None:
                g[f"sgd_{tag}_{k}_out"] = to_np(arr)

    # one MNIST-BN train step at batch 32, reduced width (config 5's network
    # shape: connected layers + BN + softmax), every buffer array checked
    widths, acts, B = [12, 8, 6, 5], [1, 0, 4], 32
    layers = []
    init = []
    for li in range(len(widths) - 1):
        I, O = widths[li], widths[li + 1]
        r = float(np.sqrt(2.0 / I))
        L = {}
        for k, n in mlp_sizes(I, O, B).items():
            if k == "W":
                arr, q = rnd(rng, n, -r, r)
            elif k == "scales":
                arr, q = rnd(rng, n, 0.8, 1.2)
            elif k in ("rmean", "b"):
                arr, q = rnd(rng, n, -0.1, 0.1)
            elif k == "rvar":
                arr, q = rnd(rng, n, 0.5, 1.5)
            elif k in ("dW", "db", "dscales"):
                arr, q = rnd(rng, n, -0.05, 0.05)   # momentum carried over from a step before
            else:
                arr, q = np.zeros(n, np.float32), [Fraction(0)] * n
            L[k] = q
            init.append(arr)
        layers.append(L)
    C = widths[-1]
    init.append(np.zeros(3 * B * C, np.float32))
    X, Xq = rnd(rng, B * widths[0], 0.0, 1.0)
    T = np.zeros(B * C, np.float32)
    T[[r * C + (r * 7 + 1) % C for r in range(B)]] = 1.0
    hyper = np.array([0.01, 0.9, 0.0005], np.float32)
    cost, sm, smd, loss = mlp_step(widths, acts, B, Xq, [F(t) for t in T], layers,
                                   *(F(t) for t in hyper))
    final = []
    for L in layers:
        for k in MLP_ORDER:
            final.append(to_np(L[k]))
    final += [to_np(sm), to_np(smd), to_np(loss)]
    g["mlp_widths"] = np.array(widths, np.int64)
    g["mlp_acts"] = np.array(acts, np.int64)
    g["mlp_B"] = np.array([B], np.int64)
    g["mlp_hyper"] = hyper
    g["mlp_X"], g["mlp_T"] = X, T
    g["mlp_buf_in"] = np.concatenate(init)
    g["mlp_buf_out"] = np.concatenate(final)
    g["mlp_cost"] = to_np([cost])

    np.savez_compressed(OUT, **g)
    print(f"wrote {OUT} ({len(g)} arrays)")


if __name__ == "__main__":
    main()
