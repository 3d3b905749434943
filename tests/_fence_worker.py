"""One rank of the failure-fence rehearsal on the CPU (tests/test_fence.py; launched by torch.distributed.run,
gloo).  Three legs shaped like the bench's N > 1 legs, every exchange through fhespear_dist.TimedDist with the
FailureFence attached exactly as bench.py attaches it:

  matvec  -- steps of local work + a gather of each rank's output to rank 0 (bench.py matvec leg);
  block   -- 4 dependent stages: rank 0 broadcasts the stage input, each rank works, the outputs come to rank 0
             point to point (tools/rwkv_block.py BlockRunner.stage);
  cfg5    -- chain blocks: a flag broadcast from rank 0, work, a reduce to rank 0, a barrier (tools/ffn_block.py
             chain_over_ranks).

FHESPEAR_BENCH_INJECT picks the failure.  Rank 0 prints one JSON line: per leg its fault (None when every rank
completed it) and its seconds; then every rank leaves through FailureFence.finish() and exits 0."""
import datetime
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "fhe-spear_amd" / "python"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import fhespear_dist as fd  # noqa: E402

WORK_S = float(os.environ.get("FENCE_WORK_S", "0.02"))
# FENCE_HANG="leg/stage@rank:seconds": that rank stalls there (outside any collective) -- a hung rank, which its own
# watcher times out after FHESPEAR_LEG_TIMEOUT seconds
_HANG = os.environ.get("FENCE_HANG", "")


def point(td, stage, rank):
    if _HANG:
        where, secs = _HANG.rsplit(":", 1)
        leg_stage, r = where.rsplit("@", 1)
        act = td.fence.active
        if act is not None and int(r) == rank and leg_stage == f"{act[1]}/{stage}":
            time.sleep(float(secs))
    td.point(stage)


def matvec_leg(td, rank, world):
    buf = torch.full((1024,), float(rank))
    for s in range(6):
        point(td, f"step{s}", rank)
        time.sleep(WORK_S)
        got = fd.gather_to_root(td, buf, world, rank)
        if rank == 0:
            assert [int(g[0]) for g in got] == list(range(world))
    return {"steps": 6}


def block_leg(td, rank, world):
    for i in range(4):
        point(td, f"stage{i}", rank)
        x = torch.full((4096,), float(i) if rank == 0 else -1.0)
        td.broadcast(x, src=0)
        assert float(x[0]) == float(i)
        time.sleep(WORK_S * (1 + rank % 2))
        if rank == 0:
            for src in range(1, world):
                y = torch.empty(4096)
                td.recv(y, src=src)
                assert float(y[0]) == i + src
        else:
            td.send(x + rank, dst=0)
    return {"stages": 4}


def cfg5_leg(td, rank, world):
    acc = torch.zeros(2048)
    for b in range(5):
        point(td, f"block{b}", rank)
        flag = torch.tensor([b % 2])
        td.broadcast(flag, src=0)
        if int(flag[0]):
            point(td, "bootstrap", rank)
        time.sleep(WORK_S)
        part = torch.full((2048,), float(rank + 1))
        td.reduce(part, dst=0)
        if rank == 0:
            acc += part
        td.barrier()
    return {"blocks": 5}


def main():
    timeout = datetime.timedelta(seconds=int(os.environ.get("FENCE_PG_TIMEOUT", "120")))
    dist.init_process_group("gloo", timeout=timeout)
    rank, world = dist.get_rank(), dist.get_world_size()

    def reinit(store):   # bench.py's: the same backend and timeout on a fresh store prefix
        dist.init_process_group("gloo", store=store, rank=rank, world_size=world, timeout=timeout)
    fence = fd.FailureFence(dist, rank, world, log=lambda m: print(m, file=sys.stderr, flush=True),
                            reinit=reinit if os.environ.get("FENCE_REINIT", "1") == "1" else None)
    td = fd.TimedDist(dist, fence)
    legs = {}
    for name, fn in (("matvec", matvec_leg), ("block", block_leg), ("cfg5", cfg5_leg)):
        t0 = time.time()
        res, fault = fence.run(name, fn, td, rank, world)
        legs[name] = {"result": res, "fault": fault, "seconds": round(time.time() - t0, 3)}
    if rank == 0:
        print(json.dumps({"world": world, "legs": legs}), flush=True)
    fence.finish()
    sys.exit(0)


if __name__ == "__main__":
    main()
