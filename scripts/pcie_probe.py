#!/usr/bin/env python3
"""Host<->device copy rates on the GPU box (sizing the host-pointer
boundary's staging): pageable vs pinned vs page-locked-in-place (hipHostRegister)
buffers, H2D and D2H alone and both directions at once, at the 64 MB operand
size of the 4096^3 SGEMM.  One JSON line.

  python scripts/pcie_probe.py
"""
import json
import time

import torch


def rate(fn, nbytes, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return round(nbytes * reps / (time.perf_counter() - t) / 1e9, 2)


def main():
    n = 16 << 20  # 64 MB of fp32
    d = torch.empty(n, device="cuda")
    d2 = torch.empty(n, device="cuda")
    page = torch.rand(n)
    page2 = torch.rand(n)
    pin = torch.rand(n).pin_memory()
    pin2 = torch.rand(n).pin_memory()
    out = {}
    out["h2d_pageable_gbs"] = rate(lambda: d.copy_(page, non_blocking=True), 4 * n)
    out["d2h_pageable_gbs"] = rate(lambda: page.copy_(d, non_blocking=True), 4 * n)
    out["h2d_pinned_gbs"] = rate(lambda: d.copy_(pin, non_blocking=True), 4 * n)
    out["d2h_pinned_gbs"] = rate(lambda: pin.copy_(d, non_blocking=True), 4 * n)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def both():
        with torch.cuda.stream(s1):
            d.copy_(pin, non_blocking=True)
        with torch.cuda.stream(s2):
            pin2.copy_(d2, non_blocking=True)
    out["bidir_pinned_gbs_total"] = rate(both, 8 * n)

    def both_page():
        with torch.cuda.stream(s1):
            d.copy_(page, non_blocking=True)
        with torch.cuda.stream(s2):
            page2.copy_(d2, non_blocking=True)
    out["bidir_pageable_gbs_total"] = rate(both_page, 8 * n)
    # page-lock the pageable buffer in place, then copy
    rt = torch.cuda.cudart()
    t = time.perf_counter()
    r = rt.cudaHostRegister(page.data_ptr(), 4 * n, 0)
    out["host_register_ms_64mb"] = round((time.perf_counter() - t) * 1e3, 3)
    out["host_register_rc"] = int(r) if not isinstance(r, tuple) else int(r[0])
    out["h2d_registered_gbs"] = rate(lambda: d.copy_(page, non_blocking=True), 4 * n)
    t = time.perf_counter()
    rt.cudaHostUnregister(page.data_ptr())
    out["host_unregister_ms_64mb"] = round((time.perf_counter() - t) * 1e3, 3)
    # host memcpy into pinned staging (single thread)
    t = time.perf_counter()
    for _ in range(5):
        pin.copy_(page)
    out["host_memcpy_to_pinned_gbs"] = round(5 * 4 * n / (time.perf_counter() - t) / 1e9, 2)
    out["torch_threads"] = torch.get_num_threads()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
