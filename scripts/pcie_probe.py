"""Host-link rates the numpy contract lives on: pinned D2H and
H2D of the per-step byte counts at 8192 envs (masks 654 MB, obs 243 MB, actions
117 MB), on one stream and split over two / four streams (several copy engines),
plus host memcpy of the action array (numpy copyto, 1 and 8 threads).

  python scripts/pcie_probe.py > gpurun_out/pcie.json
"""
import json
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        t.append(time.perf_counter() - t0)
    return round(nbytes / min(t) / 1e9, 2), round(1e3 * float(np.median(t)), 3)


def split_copy(dst, src, streams):
    k = len(streams)
    n = src.shape[0]
    cur = torch.cuda.current_stream()
    for i, s in enumerate(streams):
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            dst[i * n // k:(i + 1) * n // k].copy_(src[i * n // k:(i + 1) * n // k], non_blocking=True)
    for s in streams:
        cur.wait_stream(s)


def main():
    dev = torch.device("cuda", 0)
    out = {"device": torch.cuda.get_device_name(0)}
    sizes = {"mask_654MB": (8192, 256, 78), "obs_243MB": (8192, 256, 29), "act_117MB_i64": (8192, 256, 14)}
    streams = [torch.cuda.Stream() for _ in range(4)]
    for name, shape in sizes.items():
        d = torch.ones(shape, dtype=torch.int32, device=dev)
        h = torch.empty(shape, dtype=torch.int32, pin_memory=True)
        nb = d.numel() * 4
        r = {}
        r["d2h_1stream"] = rate(lambda: h.copy_(d, non_blocking=True), nb)
        r["d2h_2streams"] = rate(lambda: split_copy(h, d, streams[:2]), nb)
        r["d2h_4streams"] = rate(lambda: split_copy(h, d, streams), nb)
        r["h2d_1stream"] = rate(lambda: d.copy_(h, non_blocking=True), nb)
        r["h2d_2streams"] = rate(lambda: split_copy(d, h, streams[:2]), nb)
        out[name] = {"bytes": nb, **{k: {"GB/s": v[0], "ms": v[1]} for k, v in r.items()}}
    # D2H + H2D at once (full duplex)
    dm = torch.ones(sizes["mask_654MB"], dtype=torch.int32, device=dev)
    hm = torch.empty(sizes["mask_654MB"], dtype=torch.int32, pin_memory=True)
    da = torch.ones(sizes["act_117MB_i64"], dtype=torch.int32, device=dev)
    ha = torch.empty(sizes["act_117MB_i64"], dtype=torch.int32, pin_memory=True)

    def duplex():
        with torch.cuda.stream(streams[0]):
            hm.copy_(dm, non_blocking=True)
        with torch.cuda.stream(streams[1]):
            da.copy_(ha, non_blocking=True)
    out["duplex_mask_d2h_plus_act_h2d"] = rate(duplex, dm.numel() * 4 + da.numel() * 4)
    # pageable D2H (what action.cpu() does in ppo_gridnet.py:475)
    out["d2h_pageable_act"] = rate(lambda: da.cpu(), da.numel() * 4)
    # host memcpy of the action array into a pinned staging buffer
    src = np.ones((8192, 256 * 7), np.int64)
    dst = torch.empty((8192, 256 * 7), dtype=torch.int64, pin_memory=True).numpy()
    pool = ThreadPoolExecutor(8)

    def par(k):
        n = src.shape[0]
        list(pool.map(lambda i: np.copyto(dst[i * n // k:(i + 1) * n // k], src[i * n // k:(i + 1) * n // k]), range(k)))
    for k in (1, 4, 8, 16):
        t = []
        for _ in range(5):
            t0 = time.perf_counter()
            par(k)
            t.append(time.perf_counter() - t0)
        out[f"host_copyto_117MB_{k}threads"] = {"GB/s": round(src.nbytes / min(t) / 1e9, 2), "ms": round(1e3 * min(t), 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
