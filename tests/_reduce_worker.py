"""Worker of test_giant_shard.test_modular_reduce_sum_exact_beyond_int64_bound (gloo, CPU)."""
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "fhe-spear_amd" / "python"))
import fhespear_dist as fd  # noqa: E402

dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
moduli = [(1 << 60) - 93, (1 << 60) - 173, (1 << 59) - 55]          # one row per modulus
cols = 64
rng = np.random.default_rng(123)
allv = [[rng.integers(q - 2 ** 20, q, size=cols, dtype=np.uint64) for q in moduli] for _ in range(world)]
mine = torch.tensor(np.stack(allv[rank]).astype(np.int64).reshape(-1))
fd.modular_reduce_sum(dist, mine, moduli, root=0)
if rank == 0:
    ok = True
    got = mine.view(len(moduli), cols).numpy()
    for i, q in enumerate(moduli):
        for j in range(cols):
            want = sum(int(allv[r][i][j]) for r in range(world)) % q
            ok &= int(got[i, j]) == want
    print(f"reduce exact: {ok}", flush=True)
dist.destroy_process_group()
