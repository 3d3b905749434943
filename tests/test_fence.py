"""A one-rank failure ends the bench leg on every rank, on the CPU with gloo.

tests/_fence_worker.py runs three legs shaped like bench.py's N > 1 legs (a gathered matvec loop, the RWKV block's
dependent broadcast / point-to-point stages, the cfg5 chain's flag broadcast / reduce / barrier blocks) through
fhespear_dist.FailureFence + TimedDist, as bench.py does; FHESPEAR_BENCH_INJECT raises on one rank at a leg's start
or at a stage boundary while its peers wait in collectives on it.  Every configuration runs at once (distinct
ports) so the suite pays for one rendezvous."""
import json
import os
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
WORKER = REPO / "tests" / "_fence_worker.py"
LEGS = ("matvec", "block", "cfg5")

# (world, injection, re-create the process group after a failure); "hang:" = FENCE_HANG (a rank stalls outside any
# collective; FHESPEAR_LEG_TIMEOUT = 3 s makes its own watcher fail the leg)
CASES = [
    (2, "matvec/step2@1", True),
    (2, "block@0", True),
    (2, "cfg5/block3@1", True),
    (4, "matvec@2", True),
    (4, "block/stage2@1", True),
    (4, "cfg5/bootstrap@3", True),
    (4, "block/stage1@3", False),   # no re-creation: the later legs are skipped, the line still printed
    (4, "", True),                  # no failure: every leg completes, the group is destroyed cleanly
    (3, "hang:block/stage2@2:12", True),
]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def runs():
    procs = []
    for world, inj, reinit in CASES:
        env = dict(os.environ, FHESPEAR_BENCH_INJECT="" if inj.startswith("hang:") else inj,
                   FENCE_HANG=inj[5:] if inj.startswith("hang:") else "", FHESPEAR_LEG_TIMEOUT="3",
                   FENCE_REINIT="1" if reinit else "0", OMP_NUM_THREADS="1", MASTER_ADDR="127.0.0.1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", str(WORKER)]
        procs.append((time.time(), subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                                    text=True)))
    out = []
    for (world, inj, reinit), (t0, p) in zip(CASES, procs):
        try:
            so, se = p.communicate(timeout=180)
        except subprocess.TimeoutExpired:
            p.kill()
            so, se = p.communicate()
            pytest.fail(f"world {world} inject {inj!r}: hung\n{se[-3000:]}")
        line = [ln for ln in so.splitlines() if ln.startswith("{")]
        out.append(dict(world=world, inj=inj, reinit=reinit, rc=p.returncode, line=json.loads(line[-1]) if line else None,
                        stderr=se, wall=time.time() - t0))
    return out


@pytest.mark.parametrize("k", range(len(CASES)), ids=[f"w{w}-{i or 'none'}-{'reinit' if r else 'skip'}"
                                                      for w, i, r in CASES])
def test_one_rank_failure_ends_the_leg_on_every_rank(runs, k):
    r = runs[k]
    assert r["rc"] == 0, r["stderr"][-3000:]                       # torchrun: every rank exited 0, no signal
    assert "SIGTERM" not in r["stderr"] and "Signal" not in r["stderr"], r["stderr"][-3000:]
    line = r["line"]
    assert line is not None and line["world"] == r["world"], r["stderr"][-3000:]   # rank 0 printed its line
    legs = line["legs"]
    if not r["inj"]:
        assert all(legs[n]["fault"] is None for n in LEGS)
        return
    hang = r["inj"].startswith("hang:")
    where, rank = (r["inj"][5:].rsplit(":", 1)[0] if hang else r["inj"]).rsplit("@", 1)
    bad = where.split("/")[0]
    f = legs[bad]["fault"]
    assert f is not None and f["failed_ranks"] == [int(rank)], f
    assert sorted(f["abandoned_ranks"]) == [x for x in range(r["world"]) if x != int(rank)], f
    assert f["unresponsive_ranks"] == []
    if hang:   # the stalled rank's own watcher failed the leg after 3 s; its peers left then, not after the stall
        assert "still running after 3 s" in f["error"], f
        assert legs[bad]["seconds"] < 40.0, legs[bad]
    else:
        assert "injected failure" in f["error"]
        assert legs[bad]["seconds"] < 10.0, legs[bad]      # peers left the leg within seconds (gloo timeout: 120 s)
    i = LEGS.index(bad)
    for n in LEGS[:i]:
        assert legs[n]["fault"] is None, legs[n]
    for n in LEGS[i + 1:]:
        if r["reinit"]:
            assert f["process_group"].startswith("re-created")
            assert legs[n]["fault"] is None and legs[n]["result"], legs[n]   # the next legs ran on a fresh group
        else:
            assert "skipped" in legs[n]["fault"], legs[n]


def test_local_fence_reports_and_continues(monkeypatch):
    sys.path.insert(0, str(REPO / "fhe-spear_amd" / "python"))
    import fhespear_dist as fd
    monkeypatch.setenv("FHESPEAR_BENCH_INJECT", "b/s1@0")
    fence = fd.LocalFence()

    def leg_b():
        fence.point("s0")
        fence.point("s1")
        return "unreached"
    assert fence.run("a", lambda: 1) == (1, None)
    res, fault = fence.run("b", leg_b)
    assert res is None and fault["failed_ranks"] == [0] and "InjectedFailure" in fault["error"]
    assert fence.run("c", lambda: 3) == (3, None)
    assert fd.parse_inject("cfg5@3, block/stage2@1") == {("cfg5", None, 3), ("block", "stage2", 1)}
