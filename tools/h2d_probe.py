#!/usr/bin/env python3
"""Host-to-device bandwidth probe (run on the GPU box): pinned H2D of one
buffer, of the same bytes in 4/16 chunks, and the host memcpy rate into pinned
staging -- the ceilings the watch-replay pipeline (config 5) works against."""
import time

import torch

n = int(70e6)
src = torch.empty(n, dtype=torch.uint8, pin_memory=True)
src.fill_(7)
dst = torch.empty(n, dtype=torch.uint8, device="cuda")
s = torch.cuda.Stream()
for chunks in (1, 4, 16):
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        with torch.cuda.stream(s):
            for c in range(chunks):
                a, b = n * c // chunks, n * (c + 1) // chunks
                dst[a:b].copy_(src[a:b], non_blocking=True)
        s.synchronize()
        best = min(best, time.perf_counter() - t)
    print("H2D %d chunk(s): %.1f GB/s" % (chunks, n / best / 1e9))
pageable = torch.empty(n, dtype=torch.uint8)
pageable.fill_(3)
best = 1e9
for _ in range(5):
    t = time.perf_counter()
    src.copy_(pageable)
    best = min(best, time.perf_counter() - t)
print("host copy into pinned (torch, 1 call): %.1f GB/s" % (n / best / 1e9))

# the same copy while another stream keeps every CU busy (what K0 does during a batch's upload)
big = torch.empty(1 << 28, dtype=torch.float32, device="cuda")
busy = torch.cuda.Stream()
for chunks in (1, 16):
    torch.cuda.synchronize()
    with torch.cuda.stream(busy):
        for _ in range(40):
            big.mul_(1.0001)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(s):
        ev0.record(s)
        for c in range(chunks):
            a, b = n * c // chunks, n * (c + 1) // chunks
            dst[a:b].copy_(src[a:b], non_blocking=True)
        ev1.record(s)
    torch.cuda.synchronize()
    print("H2D %d chunk(s) beside a busy stream: %.1f GB/s" % (chunks, n / (ev0.elapsed_time(ev1) * 1e-3) / 1e9))

# the same bytes split over 2 / 4 copy streams at once (several SDMA engines?)
for ns in (2, 4):
    streams = [torch.cuda.Stream() for _ in range(ns)]
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(5):
        t = time.perf_counter()
        for k, st in enumerate(streams):
            a, b = n * k // ns, n * (k + 1) // ns
            with torch.cuda.stream(st):
                dst[a:b].copy_(src[a:b], non_blocking=True)
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t)
    print("H2D over %d streams: %.1f GB/s" % (ns, n / best / 1e9))
