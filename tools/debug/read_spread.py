"""Is plain streaming read bandwidth placement-dependent too?  (companion of alloc_spread.py)

A 9.66 GB int64 tensor (the size of cfg2's diagonal slab) re-allocated TRIALS times in one process, each time after
a spacer of a different size; per trial the mean time of REPS full reads (`torch.sum`) and the implied TB/s.
If this spread is small while k_bsgs_inner's is ~12 %, the Hadamard's sensitivity comes from its access pattern
(many concurrent diagonal streams), not from the memory the slab lands on.

    python tools/debug/read_spread.py [TRIALS] [REPS]
"""
import sys

import torch


def main():
    trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    n = 9663676416 // 8
    res = []
    for t in range(trials):
        spacer = torch.empty(int((0.5 + 1.7 * t) * 2 ** 30), dtype=torch.uint8, device="cuda:0")
        x = torch.ones(n, dtype=torch.int64, device="cuda:0")
        x.sum()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            s = x.sum()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        res.append(ms)
        print(f"trial {t}: spacer {spacer.numel() / 2 ** 30:.1f} GiB, read {ms:.3f} ms = {n * 8 / ms / 1e9:.2f} TB/s "
              f"(sum {int(s)})", flush=True)
        del x, spacer
        torch.cuda.empty_cache()
    print(f"streaming read over {trials} placements: min {min(res):.3f} max {max(res):.3f} ms "
          f"(spread {100 * (max(res) / min(res) - 1):.1f} %)")


if __name__ == "__main__":
    main()
