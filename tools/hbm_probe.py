"""Practical HBM rates of one MI355X for the roofline discussion: a write-only fill,
a read-only reduction and a copy, each over buffers far larger than the 256-MB Infinity Cache,
timed with HIP events over several repetitions. Prints one JSON line."""
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
    nbytes = 8 << 30
    x = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
    y = torch.empty(nbytes // 4, dtype=torch.int32, device="cuda")
    out = {}
    ms = timed(lambda: x.fill_(7))
    out["write_only_GBs"] = round(nbytes / ms / 1e6, 1)
    ms = timed(lambda: x.sum(dtype=torch.int64))
    out["read_only_GBs"] = round(nbytes / ms / 1e6, 1)
    ms = timed(lambda: y.copy_(x))
    out["copy_GBs"] = round(2 * nbytes / ms / 1e6, 1)
    out["bytes"] = nbytes
    print(json.dumps(out))


if __name__ == "__main__":
    main()
