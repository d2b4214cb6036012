"""Times nrc_sort_train_permutation (the reference's key-sort shuffle contract) on n random u32 keys: HIP events on the
stream, after warm-up; run under rocprofv3 --kernel-trace for the per-kernel split.

    python tools/time_sort.py [--n 65536 --iters 50]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import nrc_loader  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    import torch

    nrc = nrc_loader.load()
    F = nrc.frame
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    keys = torch.randint(0, 1 << 31, (args.n,), dtype=torch.int32, device=dev)
    perm = torch.empty(args.n, dtype=torch.int32, device=dev)
    temp = torch.empty(max(1, F.sort_train_permutation_temp_bytes(args.n)), dtype=torch.uint8, device=dev)
    for _ in range(5):
        F.sort_train_permutation(keys, perm, args.n, temp=temp)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.iters):
        F.sort_train_permutation(keys, perm, args.n, temp=temp)
    e1.record(stream)
    torch.cuda.synchronize()
    print(json.dumps({"n": args.n, "us_per_sort": e0.elapsed_time(e1) / args.iters * 1e3}))


if __name__ == "__main__":
    main()
