"""Darknet network description: .cfg parsing, .weights I/O, batch-norm folding
and the layer plan of a forward pass — the part of TDarknetParser / TNNet
(nparser.pas, nnet.pas) that a YOLOv3 forward needs.

* ``parse_cfg(text)``: darknet INI sections (nparser.pas:154-246 reads the
  same format through TCFGList): ``[type]`` lines, ``key=value`` options,
  ``#`` / ``;`` comments.
* ``Network(sections, batch)``: shapes of every layer exactly as the
  reference's parser derives them (nparser.pas:782-930): convolutional
  (``pad=1`` => padding = size div 2, nparser.pas:186-189; out = (in + 2p - k)
  div stride + 1, nConvolutionLayer.pas:92-100), shortcut (TAddLayer,
  naddlayer.pas), route (TConcatLayer, nconcatlayer.pas), upsample
  (TUpSampleLayer, nupsamplelayer.pas) and yolo (TYoloLayer, nyololayer.pas).
* ``load_weights`` / ``write_weights``: the darknet .weights layout read by
  TDarknetParser.loadWeights (nparser.pas:1275-1330): int32 major, minor,
  revision, then ``seen`` as uint64 when major*10+minor >= 2 (else uint32),
  then per convolutional layer biases[n], (scales, rolling_mean,
  rolling_variance)[n] when batch-normalized, weights[n*c*k*k]
  (loadConvolutionalWeights, nparser.pas:1140-1185).
* ``fuse_batchnorm``: TBaseConvolutionalLayer.fuseBatchNorm
  (nConvolutionLayer.pas:102-126) in float32: p = scale / sqrt(max(var,
  1e-6)); bias -= mean * p; W *= p.

The forward pass itself runs on the HIP backend (``HipDarknet``); the oracle
restates it on the CPU for the parity tests.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from pathlib import Path

import numpy as np

from ._abi import ACT

SEPS = np.float32(0.000001)  # sEPSILON, ntensors.pas:95


@dataclass
class Section:
    kind: str
    opts: dict = field(default_factory=dict)

    def get(self, key, default=None):
        return self.opts.get(key, default)

    def int(self, key, default=0):
        return int(self.opts.get(key, default))


def parse_cfg(text: str) -> list[Section]:
    sections: list[Section] = []
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line[0] in "#;":
            continue
        if line.startswith("["):
            sections.append(Section(line[1:line.index("]")].strip().lower()))
            continue
        if "=" not in line or not sections:
            raise ValueError(f"bad cfg line: {raw!r}")
        k, v = line.split("=", 1)
        sections[-1].opts[k.strip()] = v.strip()
    if not sections or sections[0].kind not in ("net", "network"):
        raise ValueError("1st section in config file must be a [net] parameters.")
    return sections


@dataclass
class Layer:
    index: int
    kind: str            # convolutional | shortcut | route | upsample | yolo
    c: int               # input channels / height / width
    h: int
    w: int
    out_c: int
    out_h: int
    out_w: int
    filters: int = 0
    size: int = 1
    stride: int = 1
    pad: int = 0
    activation: int = ACT["LINEAR"]
    bn: bool = False
    inputs: tuple = ()   # shortcut: (from,), route: the layers, others: ()
    anchors: int = 0     # yolo: anchors of this scale (len(mask))
    classes: int = 0

    @property
    def out_size(self) -> int:
        return self.out_c * self.out_h * self.out_w


def _act(name: str) -> int:
    return ACT[name.strip().upper()]


class Network:
    """Layer plan with shapes (nparser.pas:782-930)."""

    def __init__(self, sections: list[Section], batch: int | None = None):
        net = sections[0]
        self.batch = batch if batch is not None else net.int("batch", 1)
        self.h, self.w, self.c = net.int("height"), net.int("width"), net.int("channels", 3)
        self.layers: list[Layer] = []
        c, h, w = self.c, self.h, self.w
        for sec in sections[1:]:
            i = len(self.layers)
            if sec.kind in ("convolutional", "conv"):
                size = sec.int("size", 1)
                stride = sec.int("stride", 1)
                pad = size // 2 if sec.int("pad", 0) else sec.int("padding", 0)
                f = sec.int("filters", 1)
                oh = (h + 2 * pad - size) // stride + 1
                ow = (w + 2 * pad - size) // stride + 1
                lay = Layer(i, "convolutional", c, h, w, f, oh, ow, filters=f, size=size,
                            stride=stride, pad=pad, activation=_act(sec.get("activation", "logistic")),
                            bn=bool(sec.int("batch_normalize", 0)))
            elif sec.kind == "shortcut":
                src = int(sec.get("from"))
                src = src + i if src < 0 else src
                lay = Layer(i, "shortcut", c, h, w, c, h, w,
                            activation=_act(sec.get("activation", "linear")), inputs=(src,))
            elif sec.kind in ("route", "concat"):
                srcs = tuple(int(v) + i if int(v) < 0 else int(v)
                             for v in sec.get("layers").split(","))
                first = self.layers[srcs[0]]
                oc = sum(self.layers[s].out_c for s in srcs)
                lay = Layer(i, "route", c, h, w, oc, first.out_h, first.out_w, inputs=srcs)
            elif sec.kind == "upsample":
                s = sec.int("stride", 2)
                lay = Layer(i, "upsample", c, h, w, c, h * s, w * s, stride=s)
            elif sec.kind == "yolo":
                mask = [m for m in sec.get("mask", "").split(",") if m.strip()]
                classes = sec.int("classes", 20)
                lay = Layer(i, "yolo", c, h, w, c, h, w, anchors=len(mask), classes=classes)
                if c != len(mask) * (classes + 5):
                    raise ValueError(f"yolo layer {i}: {c} channels for {len(mask)} anchors")
            else:
                raise ValueError(f"[Parser][{sec.kind}] layer is not yet implemented!")
            self.layers.append(lay)
            c, h, w = lay.out_c, lay.out_h, lay.out_w

    def convs(self) -> list[Layer]:
        return [l for l in self.layers if l.kind == "convolutional"]


def yolov3_cfg(size: int = 416, batch: int = 1, classes: int = 80) -> str:
    """The darknet YOLOv3 network (the public yolov3.cfg structure; the
    reference loads that file from outside its tree, MSCOCOYolo.pas:28-34)."""
    out = [f"[net]\nbatch={batch}\nsubdivisions=1\nwidth={size}\nheight={size}\nchannels=3\n"]

    def conv(f, k, s=1, act="leaky", bn=True):
        out.append(f"[convolutional]\n{'batch_normalize=1' + chr(10) if bn else ''}"
                   f"filters={f}\nsize={k}\nstride={s}\npad=1\nactivation={act}\n")

    def res(n, c):
        for _ in range(n):
            conv(c // 2, 1)
            conv(c, 3)
            out.append("[shortcut]\nfrom=-3\nactivation=linear\n")

    anchors = "10,13, 16,30, 33,23, 30,61, 62,45, 59,119, 116,90, 156,198, 373,326"

    def yolo(mask):
        out.append(f"[yolo]\nmask = {mask}\nanchors = {anchors}\nclasses={classes}\nnum=9\n"
                   "jitter=.3\nignore_thresh = .7\ntruth_thresh = 1\nrandom=1\n")

    det = 3 * (classes + 5)
    conv(32, 3)
    conv(64, 3, 2); res(1, 64)
    conv(128, 3, 2); res(2, 128)
    conv(256, 3, 2); res(8, 256)
    conv(512, 3, 2); res(8, 512)
    conv(1024, 3, 2); res(4, 1024)
    for _ in range(2):
        conv(512, 1); conv(1024, 3)
    conv(512, 1); conv(1024, 3); conv(det, 1, act="linear", bn=False)
    yolo("6,7,8")
    out.append("[route]\nlayers = -4\n")
    conv(256, 1)
    out.append("[upsample]\nstride=2\n")
    out.append("[route]\nlayers = -1, 61\n")
    for _ in range(2):
        conv(256, 1); conv(512, 3)
    conv(256, 1); conv(512, 3); conv(det, 1, act="linear", bn=False)
    yolo("3,4,5")
    out.append("[route]\nlayers = -4\n")
    conv(128, 1)
    out.append("[upsample]\nstride=2\n")
    out.append("[route]\nlayers = -1, 36\n")
    for _ in range(3):
        conv(128, 1); conv(256, 3)
    conv(det, 1, act="linear", bn=False)
    yolo("0,1,2")
    return "\n".join(out)


# ---- parameters -------------------------------------------------------------

@dataclass
class ConvParams:
    biases: np.ndarray
    weights: np.ndarray                 # [filters][c*k*k]
    scales: np.ndarray | None = None    # batch norm (before folding)
    rolling_mean: np.ndarray | None = None
    rolling_var: np.ndarray | None = None


def random_params(net: Network, seed: int = 3) -> list[ConvParams]:
    """Synthetic parameters of the reference's initialisation scale
    (nConvolutionLayer.pas:216-220: U[-s, s], s = sqrt(2/(k*k*c)))."""
    rng = np.random.default_rng(seed)
    ps = []
    for l in net.convs():
        s = np.sqrt(2.0 / (l.size * l.size * l.c))
        w = rng.uniform(-s, s, (l.filters, l.c * l.size * l.size)).astype(np.float32)
        b = rng.uniform(-0.1, 0.1, l.filters).astype(np.float32)
        if l.bn:
            ps.append(ConvParams(b, w, rng.uniform(0.5, 1.5, l.filters).astype(np.float32),
                                 rng.uniform(-0.1, 0.1, l.filters).astype(np.float32),
                                 rng.uniform(0.5, 2.0, l.filters).astype(np.float32)))
        else:
            ps.append(ConvParams(b, w))
    return ps


def write_weights(path, net: Network, params: list[ConvParams], major=0, minor=2, revision=0,
                  seen=0) -> None:
    with open(path, "wb") as f:
        f.write(struct.pack("<3i", major, minor, revision))
        f.write(struct.pack("<Q" if major * 10 + minor >= 2 else "<I", seen))
        for l, p in zip(net.convs(), params):
            f.write(p.biases.astype("<f4").tobytes())
            if l.bn:
                for t in (p.scales, p.rolling_mean, p.rolling_var):
                    f.write(t.astype("<f4").tobytes())
            f.write(p.weights.astype("<f4").tobytes())


def load_weights(path, net: Network) -> tuple[list[ConvParams], int]:
    """Returns the per-conv parameters and ``seen``."""
    data = Path(path).read_bytes()
    major, minor, _rev = struct.unpack_from("<3i", data, 0)
    off = 12
    if major * 10 + minor >= 2:
        (seen,) = struct.unpack_from("<Q", data, off)
        off += 8
    else:
        (seen,) = struct.unpack_from("<I", data, off)
        off += 4

    def take(n):
        nonlocal off
        if off + 4 * n > len(data):
            raise ValueError("Unexpected end of weights-file")
        a = np.frombuffer(data, "<f4", n, off).astype(np.float32)
        off += 4 * n
        return a

    ps = []
    for l in net.convs():
        b = take(l.filters)
        sc = rm = rv = None
        if l.bn:
            sc, rm, rv = take(l.filters), take(l.filters), take(l.filters)
        w = take(l.filters * l.c * l.size * l.size).reshape(l.filters, -1)
        ps.append(ConvParams(b, w, sc, rm, rv))
    return ps, seen


def fuse_batchnorm(l: Layer, p: ConvParams) -> ConvParams:
    """fuseBatchNorm (nConvolutionLayer.pas:102-126), float32 throughout."""
    if not l.bn:
        return ConvParams(p.biases.copy(), p.weights.copy())
    pre = (p.scales / np.sqrt(np.maximum(p.rolling_var, SEPS))).astype(np.float32)
    b = (p.biases - (p.rolling_mean * pre).astype(np.float32)).astype(np.float32)
    w = (p.weights * pre[:, None]).astype(np.float32)
    return ConvParams(b, w)


class HipDarknet:
    """TNNet.forward over a darknet layer plan on the HIP backend (nnet.pas:
    275-310 selects forwardGPU per layer): every layer's output stays in a
    device buffer of its own; convolutions take BN-folded parameters
    (fuseBatchNorm) and run the fused implicit-GEMM driver."""

    def __init__(self, hip, net: Network, params: list[ConvParams], torch):
        self.hip, self.net, self.torch = hip, net, torch
        B = net.batch
        dev = "cuda"
        self.out = [torch.empty(B * l.out_size, device=dev) for l in net.layers]
        self.conv_params = {}
        for l, p in zip(net.convs(), params):
            f = fuse_batchnorm(l, p)
            self.conv_params[l.index] = (torch.from_numpy(np.ascontiguousarray(f.weights)).to(dev),
                                         torch.from_numpy(np.ascontiguousarray(f.biases)).to(dev))

    def forward(self, x):
        """x: device tensor [batch, c, h, w] (contiguous).  Returns the per-
        layer output buffers (the yolo layers' are the detections)."""
        hip, B = self.hip, self.net.batch
        prev = x
        for l in self.net.layers:
            out = self.out[l.index]
            if l.kind == "convolutional":
                w, b = self.conv_params[l.index]
                hip.convForward(B, l.c, l.h, l.w, prev, w, b, l.filters, l.size, l.stride, l.pad,
                                1, l.activation, None, out, fused=True)
            elif l.kind == "shortcut":
                src = self.out[l.inputs[0]]
                hip.shortcut(B * l.out_size, prev, 0, src, 0, out, 0, l.activation)
            elif l.kind == "route":  # TTensor.concat: whole tensors in order
                off = 0
                for s in l.inputs:
                    n = B * self.net.layers[s].out_size
                    hip.copy(n, self.out[s], 0, 1, out, off, 1)
                    off += n
            elif l.kind == "upsample":
                hip.upSample(B, l.c, l.h, l.w, prev, l.stride, 1, 1.0, out)
            elif l.kind == "yolo":
                hip.yoloForward(B, l.anchors, l.classes, l.h * l.w, prev, out)
            prev = out
        return self.out


class HipDarknetTrain:
    """One training pass of a darknet network on the HIP backend, in the
    reference's call order: TNet.forward in training (nnet.pas:275-322; each
    layer's delta zeroed by ``cuda.scale(size, 0, delta, 1)`` before its
    forward) and TNet.backward (nnet.pas:323-366: layers from the last to the
    first, layer i's state.delta = layer i-1's delta, none for layer 0),
    each layer through the TNNHip call its backwardGPU makes:

    * convolutional: ``convBackwardBN`` (batch-normalized layers:
      Derivative + batchNormBack + dW + state.delta, nConvolutionLayer.pas:
      571-671 -> nbaselayer.pas:372-395) or ``convBackward`` (the 1x1
      detection heads: Derivative + addSums + dW + state.delta);
    * shortcut (TAddLayer.backwardGPU, naddlayer.pas:924-949): DeriveArray,
      then ``addvv`` of its delta into state.delta and into the from-layer's
      delta;
    * route (TConcatLayer.backwardGPU, nconcatlayer.pas:234-256): ``addvv`` of
      its delta slices into each input layer's delta;
    * upsample (TUpSampleLayer.backwardGPU, nupsamplelayer.pas:214-228):
      ``upSample(..., isForward = 0)`` accumulating into state.delta;
    * yolo (TYoloLayer.backwardGPU, nyololayer.pas:1112-1125): ``axpy`` of its
      delta (scaled by lossScale*deltaNormalizer) into state.delta.  The yolo
      loss that fills that delta during the training forward is out of scope
      (DESIGN.md); ``set_yolo_deltas`` supplies it.

    Convolutions with batch norm run ``convForwardTrain`` (training-time BN,
    nbaselayer.pas:336-370) in the forward, the heads ``convForward``.  No
    weight update is made here (TNet.update is a separate call per layer,
    ``sgdUpdate``)."""

    def __init__(self, hip, net: Network, params: list[ConvParams], torch, loss_scale: float = 1.0):
        self.hip, self.net, self.torch = hip, net, torch
        self.loss_scale = float(loss_scale)
        B = net.batch
        dev = "cuda"
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32)).to(dev)  # noqa: E731
        self.out = [torch.zeros(B * l.out_size, device=dev) for l in net.layers]
        self.delta = [torch.zeros(B * l.out_size, device=dev) for l in net.layers]
        self.conv = {}
        ws = 1
        for l, p in zip(net.convs(), params):
            n = B * l.out_size
            st = {"w": t(p.weights), "b": t(p.biases),
                  "wu": torch.zeros(p.weights.size, device=dev),
                  "bu": torch.zeros(l.filters, device=dev)}
            if l.bn:
                st.update(scales=t(p.scales), rm=t(p.rolling_mean), rv=t(p.rolling_var),
                          mean=torch.zeros(l.filters, device=dev),
                          var=torch.zeros(l.filters, device=dev),
                          x=torch.zeros(n, device=dev), xn=torch.zeros(n, device=dev),
                          su=torch.zeros(l.filters, device=dev),
                          md=torch.zeros(l.filters, device=dev),
                          vd=torch.zeros(l.filters, device=dev))
            self.conv[l.index] = st
            ws = max(ws, B * l.c * l.size * l.size * l.out_h * l.out_w)
        self.ws = torch.empty(ws, device=dev)

    def forward(self, x):
        """TNet.forward with state.isTraining (BN statistics of the batch,
        rolling statistics updated with bnMomentum 0.1)."""
        hip, B = self.hip, self.net.batch
        prev = x
        for l in self.net.layers:
            hip.scale(self.delta[l.index].numel(), 0.0, self.delta[l.index], 1)
            out = self.out[l.index]
            if l.kind == "convolutional":
                st = self.conv[l.index]
                if l.bn:
                    hip.convForwardTrain(B, l.c, l.h, l.w, prev, st["w"], l.filters, l.size,
                                         l.stride, l.pad, 1, l.activation, st["scales"], st["b"],
                                         st["rm"], st["rv"], 0.1, True, st["mean"], st["var"],
                                         st["x"], st["xn"], self.ws, out)
                else:
                    hip.convForward(B, l.c, l.h, l.w, prev, st["w"], st["b"], l.filters, l.size,
                                    l.stride, l.pad, 1, l.activation, self.ws, out, fused=True)
            elif l.kind == "shortcut":
                hip.shortcut(B * l.out_size, prev, 0, self.out[l.inputs[0]], 0, out, 0,
                             l.activation)
            elif l.kind == "route":
                off = 0
                for s in l.inputs:
                    n = B * self.net.layers[s].out_size
                    hip.copy(n, self.out[s], 0, 1, out, off, 1)
                    off += n
            elif l.kind == "upsample":
                hip.upSample(B, l.c, l.h, l.w, prev, l.stride, 1, 1.0, out)
            elif l.kind == "yolo":
                hip.yoloForward(B, l.anchors, l.classes, l.h * l.w, prev, out)
            prev = out
        return self.out

    def set_yolo_deltas(self, deltas):
        """The yolo layers' deltas (what their training forward's loss would
        leave), in layer order."""
        ys = [l for l in self.net.layers if l.kind == "yolo"]
        for l, d in zip(ys, deltas):
            self.delta[l.index].copy_(d.reshape(-1))

    def backward(self, x, on_backward=None):
        """TNet.backward (nnet.pas:323-366) over every layer; on_backward(l)
        after each layer's calls (TNet.OnBackward, nnet.pas:361-362)."""
        hip, B, L = self.hip, self.net.batch, self.net.layers
        for l in reversed(L):
            i = l.index
            inp = x if i == 0 else self.out[i - 1]
            sd = None if i == 0 else self.delta[i - 1]
            d = self.delta[i]
            if l.kind == "convolutional":
                st = self.conv[i]
                if l.bn:
                    hip.convBackwardBN(B, l.c, l.h, l.w, inp, st["w"], l.filters, l.size,
                                       l.stride, l.pad, 1, l.activation, self.out[i], d,
                                       st["scales"], st["x"], st["xn"], st["mean"], st["var"],
                                       st["su"], st["md"], st["vd"], st["wu"], self.ws, sd)
                else:
                    hip.convBackward(B, l.c, l.h, l.w, inp, st["w"], l.filters, l.size, l.stride,
                                     l.pad, 1, l.activation, self.out[i], d, st["bu"], st["wu"],
                                     self.ws, sd)
            elif l.kind == "shortcut":
                n = d.numel()
                hip.DeriveArray(n, self.out[i], 0, l.activation, d)
                hip.addvv(n, d, 0, 1, sd, 0, 1, sd, 0, 1)
                src = self.delta[l.inputs[0]]
                hip.addvv(n, src, 0, 1, d, 0, 1, src, 0, 1)
            elif l.kind == "route":
                off = 0
                for s in l.inputs:
                    pt = self.delta[s]
                    hip.addvv(pt.numel(), pt, 0, 1, d, off, 1, pt, 0, 1)
                    off += pt.numel()
            elif l.kind == "upsample":
                hip.upSample(B, l.c, l.h, l.w, sd, l.stride, 0, 1.0, d)
            elif l.kind == "yolo":
                hip.axpy(sd.numel(), self.loss_scale, d, 0, 1, sd, 0, 1)
            if on_backward is not None:
                on_backward(l)
