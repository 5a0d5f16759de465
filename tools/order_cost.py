#!/usr/bin/env python3
"""What ordering a batch's singleton packets by CT home bucket would cost per step
("config 3 address order"): a full radix sort of 14M 64-bit keys
{bucket << 32 | packet} and a one-pass counting sort by the bucket's top 16 bits (the
near-ascending order that binning gives), timed on the GPU with HIP events.  The gain
is bounded by the stage's CT bucket reads (tools/tlb_probe.py: ascending lines ran 2.5x
the random rate at 32 GiB).  Prints one JSON line."""
import json
import torch


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    n = 14_000_000                                                # config 3's singletons per 2^24-packet step
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(7)
    bucket = torch.randint(0, 1 << 27, (n,), device=dev, generator=g, dtype=torch.int64)
    keys = (bucket << 32) | torch.arange(n, device=dev, dtype=torch.int64)
    sort_ms = timed(lambda: torch.sort(keys))
    top = (bucket >> 11).to(torch.int32)                          # 2^16 bins of 2^11 buckets

    def bin_sort():
        cnt = torch.bincount(top, minlength=1 << 16)
        off = torch.cumsum(cnt, 0) - cnt
        order = torch.argsort(top, stable=False)                  # (torch has no scatter-by-bin; an upper bound)
        return off, order
    bin_ms = timed(bin_sort)
    hist_ms = timed(lambda: torch.bincount(top, minlength=1 << 16))
    print(json.dumps({"keys": n, "radix_sort_ms": round(sort_ms, 3), "bin_argsort_ms": round(bin_ms, 3),
                      "histogram_ms": round(hist_ms, 3)}))


if __name__ == "__main__":
    main()
