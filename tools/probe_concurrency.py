"""Diagnostic: do two HIP streams run kernels concurrently on this box?"""
import time

import torch

dev = torch.device("cuda:0")
a, b = torch.cuda.Stream(), torch.cuda.Stream()
x = torch.empty(256 * 1024 * 1024 // 4, device=dev)  # 256 MiB
y = torch.empty_like(x)


def timeit(fn, n=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


CY = 2_000_000
print("sleep alone", timeit(lambda: torch.cuda._sleep(CY)))


def two_sleeps():
    with torch.cuda.stream(a):
        torch.cuda._sleep(CY)
    with torch.cuda.stream(b):
        torch.cuda._sleep(CY)


print("two sleeps, two streams", timeit(two_sleeps))


def copies():
    for _ in range(4):
        y.copy_(x)


print("4 copies alone", timeit(copies))


def copies_and_sleeps():
    with torch.cuda.stream(a):
        copies()
    with torch.cuda.stream(b):
        for _ in range(40):
            torch.cuda._sleep(CY // 40)


print("sleeps alone(40 small)", timeit(lambda: [torch.cuda._sleep(CY // 40) for _ in range(40)]))
print("copies || 40 small sleeps", timeit(copies_and_sleeps))
