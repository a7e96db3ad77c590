"""Streaming write / read / copy rates on the GPU for buffers inside and outside
the 256 MiB Infinity Cache (calibration for the rollout's recorded outputs).

python tools/hbm_probe.py
"""
import torch


def rate(fn, nbytes, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return nbytes * iters / (e0.elapsed_time(e1) / 1e3) / 1e9


def main():
    for mb in (64, 2048):
        n = mb * (1 << 20) // 4
        a = torch.empty(n, device="cuda")
        b = torch.empty(n, device="cuda")
        a.fill_(1.0)
        print(f"{mb:5d} MiB  write (fill_) {rate(lambda: b.fill_(2.0), 4 * n):8.0f} GB/s   "
              f"read (sum) {rate(lambda: a.sum(), 4 * n):8.0f} GB/s   "
              f"copy (r+w) {rate(lambda: b.copy_(a), 8 * n):8.0f} GB/s", flush=True)
        del a, b


if __name__ == "__main__":
    main()
