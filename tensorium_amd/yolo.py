"""YOLOv3-416 convolution workload and the conv-layer driver.

``yolov3_conv_table()`` rebuilds the 75 ``[convolutional]`` sections of the
public darknet yolov3.cfg (the cfg itself is not in the reference repo —
Samples/FPC/MSCOCO_Yolo/MSCOCOYolo.pas:28-34 loads it from outside), using the
reference's layer arithmetic: ``pad=1 ⇒ padding = size div 2``
(nparser.pas:186-189) and ``out = (in + 2p − k) div s + 1``
(nConvolutionLayer.pas:92-100).  Shortcut / route / upsample / yolo layers
are not convolutions and are outside the hot path; the table records the
shapes they produce so every conv gets its exact input shape.

``ConvolutionalLayer`` mirrors TConvolutionalLayer's forward on the HIP
backend (nConvolutionLayer.pas:457-569 CPU / 1022-1153 GPU): Conv2D → bias
(BN folded by fuseBatchNorm, 102-126) → activation.
"""
from __future__ import annotations

from dataclasses import dataclass

from ._abi import ACT


@dataclass(frozen=True)
class ConvSpec:
    index: int          # conv ordinal 0..74
    c: int              # input channels
    h: int              # input height (= width)
    filters: int
    size: int           # kernel size
    stride: int
    pad: int            # padding (size div 2)
    activation: int     # TActivationType ordinal
    batch_normalize: bool

    @property
    def out_h(self) -> int:
        return (self.h + 2 * self.pad - self.size) // self.stride + 1

    @property
    def M(self) -> int:
        return self.filters

    @property
    def N(self) -> int:
        return self.out_h * self.out_h

    @property
    def K(self) -> int:
        return self.c * self.size * self.size

    @property
    def flops(self) -> int:
        return 2 * self.M * self.N * self.K

    @property
    def needs_im2col(self) -> bool:
        # ntensors.pas:8286-8288
        return self.size != 1 or self.stride != 1

    @property
    def col_elems(self) -> int:
        return self.K * self.N if self.needs_im2col else 0


def yolov3_conv_table(size: int = 416) -> list[ConvSpec]:
    specs: list[ConvSpec] = []
    state = {"c": 3, "h": size}

    def conv(filters, k, s=1, act="LEAKY", bn=True, src=None):
        c, h = src if src is not None else (state["c"], state["h"])
        spec = ConvSpec(len(specs), c, h, filters, k, s, k // 2, ACT[act], bn)
        specs.append(spec)
        state["c"], state["h"] = filters, spec.out_h
        return (filters, spec.out_h)

    def res(n):
        for _ in range(n):
            c = state["c"]
            conv(c // 2, 1)
            conv(c, 3)   # shortcut add keeps (c, h)

    conv(32, 3)
    conv(64, 3, 2); res(1)
    conv(128, 3, 2); res(2)
    conv(256, 3, 2); res(8)
    r36 = (state["c"], state["h"])
    conv(512, 3, 2); res(8)
    r61 = (state["c"], state["h"])
    conv(1024, 3, 2); res(4)
    # head 1 @13
    conv(512, 1); conv(1024, 3); conv(512, 1); conv(1024, 3)
    route1 = conv(512, 1)
    conv(1024, 3); conv(255, 1, act="LINEAR", bn=False)
    conv(256, 1, src=route1)
    state["c"], state["h"] = 256 + r61[0], r61[1]          # upsample x2 + concat
    # head 2 @26
    conv(256, 1); conv(512, 3); conv(256, 1); conv(512, 3)
    route2 = conv(256, 1)
    conv(512, 3); conv(255, 1, act="LINEAR", bn=False)
    conv(128, 1, src=route2)
    state["c"], state["h"] = 128 + r36[0], r36[1]
    # head 3 @52
    conv(128, 1); conv(256, 3); conv(128, 1); conv(256, 3); conv(128, 1); conv(256, 3)
    conv(255, 1, act="LINEAR", bn=False)
    assert len(specs) == 75, len(specs)
    return specs


def yolov3_gflop_per_image(size: int = 416) -> float:
    return sum(s.flops for s in yolov3_conv_table(size)) / 1e9
