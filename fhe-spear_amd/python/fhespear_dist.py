"""Multi-GPU plumbing for the 8-projection RWKV block (BASELINE configs[3]/[4]).

One process per GPU (torchrun); backend "nccl" = RCCL over xGMI on MI355X, "gloo" in CPU tests.
The data path has exactly two exchange steps, both on flat int64 views of ciphertext limbs:

  * gather_to_root   -- every rank's output ciphertext(s) to rank 0 (the "client" decrypts there);
  * broadcast_from   -- one rank's ciphertext limbs to all: the stage inputs from the client, and
                        (BlockRunner baby_mode="broadcast") the G baby steps of an input that several
                        ranks need, e.g. the FFN key pair, bg:563, north_star "computed once and
                        broadcast".

Projections are assigned round-robin (projection p -> rank p % world).  The reference runs the
block's 8 BSGS calls serially in one process (bg:784-892); which of them are independent:
r, k, v (same input x) -> o -> ffn key pair (shared input, shared baby steps) -> ffn value pair.

Latency mode: one matvec's B giant groups split over the ranks
(`giant_groups`); each rank computes its groups' rotated inner sums without the rescale
(`bsgs_giant_partial`, one fused linear transform), the partial ciphertexts are summed mod q_i on
the root (`modular_reduce_sum`: RCCL int64 sum, then one reduction) and the root rescales.  Every
giant term is an exact residue (the library sums giant steps before ModDown exactly), so the result
is limb-identical to the one-GPU fused BSGS.
"""
from __future__ import annotations

# block stage structure of bg.client_aided_block (bg:784-892): projections per stage
RWKV_BLOCK_STAGES = (("r", "k", "v"), ("o",), ("ffn_key_0", "ffn_key_1"), ("ffn_val_0", "ffn_val_1"))
RWKV_BLOCK_PROJECTIONS = tuple(p for st in RWKV_BLOCK_STAGES for p in st)
# projections of one stage that take the same input ciphertext, hence the same baby steps (bg:563)
RWKV_SHARED_INPUTS = (("ffn_key_0", "ffn_key_1"),)


class TimedDist:
    """torch.distributed with every data-path exchange logged (VERDICT r4 missing #4: the N > 1 line must
    separate RCCL broadcast / gather / reduce / reduce-scatter / send-recv time from compute).  Pass it
    wherever a `dist` module is taken (BlockRunner, FfnRanks, the bench's gather); everything else is
    delegated.  Per call: kind, bytes moved by this rank's tensor, and its duration -- for device tensors a
    pair of HIP events on the current stream around the collective (torch makes that stream wait for the
    RCCL stream, so the pair brackets the transfer and the wait for the peers, without synchronising the
    host); for host tensors (gloo) wall time.  Calls moving < 4 KiB (headers) are logged as `<kind>_small`;
    object and barrier collectives as `all_gather_object` / `barrier` (bytes 0).
    With a FailureFence attached (`fence`), every collective first checks that no peer has failed in the
    running leg, and `point(stage)` marks a stage boundary of a leg (fence check + failure injection)."""

    KINDS = ("broadcast", "gather", "reduce", "reduce_scatter", "all_reduce", "send", "recv", "all_gather",
             "all_gather_object", "barrier")

    def __init__(self, dist, fence=None):
        self._d = dist
        self.fence = fence
        self.on = False
        self.log = []

    def __getattr__(self, name):
        return getattr(self._d, name)

    def start(self):
        self.log, self.on = [], True

    def stop(self):
        self.on = False

    def point(self, stage):
        if self.fence is not None:
            self.fence.point(stage)

    def _timed(self, kind, tensor, fn, *a, **k):
        if self.fence is not None:
            self.fence.check()
            self.fence.waiting = True   # a leg timeout that fires now is a peer's stall, not this rank's
            try:
                return self._timed_call(kind, tensor, fn, *a, **k)
            finally:
                self.fence.waiting = False
        return self._timed_call(kind, tensor, fn, *a, **k)

    def _timed_call(self, kind, tensor, fn, *a, **k):
        if not self.on:
            return fn(*a, **k)
        import time
        import torch
        nbytes = tensor.numel() * tensor.element_size() if tensor is not None else 0
        if nbytes < 4096 and tensor is not None:
            kind += "_small"
        if tensor is not None and tensor.is_cuda:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **k)
            e1.record()
            self.log.append((kind, nbytes, (e0, e1)))
        else:
            t0 = time.perf_counter()
            r = fn(*a, **k)
            self.log.append((kind, nbytes, time.perf_counter() - t0))
        return r

    def broadcast(self, tensor, *a, **k):
        return self._timed("broadcast", tensor, self._d.broadcast, tensor, *a, **k)

    def gather(self, tensor, *a, **k):
        return self._timed("gather", tensor, self._d.gather, tensor, *a, **k)

    def reduce(self, tensor, *a, **k):
        return self._timed("reduce", tensor, self._d.reduce, tensor, *a, **k)

    def all_reduce(self, tensor, *a, **k):
        return self._timed("all_reduce", tensor, self._d.all_reduce, tensor, *a, **k)

    def reduce_scatter_tensor(self, out, inp, *a, **k):
        return self._timed("reduce_scatter", inp, self._d.reduce_scatter_tensor, out, inp, *a, **k)

    def all_gather(self, outs, tensor, *a, **k):
        return self._timed("all_gather", tensor, self._d.all_gather, outs, tensor, *a, **k)

    def all_gather_object(self, outs, obj, *a, **k):
        return self._timed("all_gather_object", None, self._d.all_gather_object, outs, obj, *a, **k)

    def barrier(self, *a, **k):
        return self._timed("barrier", None, self._d.barrier, *a, **k)

    def send(self, tensor, *a, **k):
        return self._timed("send", tensor, self._d.send, tensor, *a, **k)

    def recv(self, tensor, *a, **k):
        return self._timed("recv", tensor, self._d.recv, tensor, *a, **k)

    def summary(self, per=1):
        """{kind: {calls, MB, ms}} over the logged calls, divided by `per` (e.g. the timed steps); call after
        the device work is complete (the events are read)."""
        import torch
        if any(isinstance(v, tuple) for _, _, v in self.log):
            torch.cuda.synchronize()
        out = {}
        for kind, nbytes, v in self.log:
            ms = v[0].elapsed_time(v[1]) if isinstance(v, tuple) else 1e3 * v
            s = out.setdefault(kind, {"calls": 0, "MB": 0.0, "ms": 0.0})
            s["calls"] += 1
            s["MB"] += nbytes / 1e6
            s["ms"] += ms
        return {k: {"calls": round(v["calls"] / per, 2), "MB": round(v["MB"] / per, 3), "ms": round(v["ms"] / per, 3)}
                for k, v in sorted(out.items())}


# ------------------------------------------------------------------ failure agreement (bench legs over N ranks)
class PeerFailed(RuntimeError):
    """Raised on a rank whose leg is abandoned because another rank failed in it."""


class InjectedFailure(RuntimeError):
    """The failure FHESPEAR_BENCH_INJECT asked for (tests of the fence)."""


def parse_inject(spec):
    """FHESPEAR_BENCH_INJECT = "leg[/stage]@rank[,...]": raise InjectedFailure on that rank when leg `leg` starts
    (no stage) or reaches FailureFence.point(stage).  Returns {(leg, stage or None, rank)}."""
    out = set()
    for item in (spec or "").split(","):
        item = item.strip()
        if not item:
            continue
        where, rank = item.rsplit("@", 1)
        leg, _, stage = where.partition("/")
        out.add((leg, stage or None, int(rank)))
    return out


class FailureFence:
    """One rank's failure ends the leg on every rank, within seconds.

    A bench run at N ranks is a sequence of legs (matvec, SEAL, RWKV block, cfg5 chain...).  Each runs through
    `run(name, fn)`.  The agreement goes through the c10d store, never through the process group the legs'
    collectives use, so it works while a peer sits in a collective:
      * a rank whose leg raises publishes the error under the leg's `fail` key and aborts its process group
        (gloo closes its pairs, so peers blocked on this rank wake at once; RCCL aborts its communicators);
      * every rank runs a watcher thread that polls that key while a leg runs; on a peer's failure it aborts its
        own process group, which wakes a collective this rank is blocked in, and `check()` / `point()` raise
        PeerFailed at the next collective or stage boundary (TimedDist calls check() before every collective);
      * at the leg's end every rank publishes {ok, error} and waits (polling, bounded) for all ranks' statuses:
        all ranks then return the same verdict -- None, or {"error", "failed_ranks", "abandoned_ranks",
        "unresponsive_ranks"};
      * a leg that failed may leave collectives half-issued, so the process group is aborted on every rank;
        with `reinit` (a function of a c10d store that makes a new default process group) every rank then joins
        a fresh one under a new store prefix and the next leg runs; without it, or when a rank did not report,
        the later legs are skipped (`run` returns {"skipped": ...}); `finish()` lets rank 0 print its line
        before the others exit, and destroys the process group when it is still intact.
    A leg still running after `leg_timeout_s` counts as failed on that rank -- after twice that while the rank waits
    inside a collective (TimedDist sets `waiting`), so the rank that stalls elsewhere is the one named.
    World 1 without a process group: LocalFence (the same interface, legs independent)."""

    PREFIX = "fhespear_fence/"

    def __init__(self, dist, rank, world, store=None, poll_s=0.1, agree_timeout_s=300.0, leg_timeout_s=None,
                 inject=None, log=None, reinit=None, max_reinits=3):
        import os
        import threading
        self.d, self.rank, self.world = dist, rank, world
        self.store = store if store is not None else dist.distributed_c10d._get_default_store()
        self.poll_s, self.agree_timeout_s = poll_s, agree_timeout_s
        self.leg_timeout_s = leg_timeout_s if leg_timeout_s is not None else float(
            os.environ.get("FHESPEAR_LEG_TIMEOUT", "1200"))
        self.inject = parse_inject(os.environ.get("FHESPEAR_BENCH_INJECT")) if inject is None else set(inject)
        self.log = log or (lambda m: None)
        self.seq = 0
        self.active = None        # (seq, name, start time) of the running leg
        self.tripped = None       # a peer's failure message for the running leg
        self.aborted = False      # process group aborted: no collective may follow
        self.waiting = False      # inside a collective (TimedDist)
        self.failed_leg = None
        self.reinit, self.reinits_left, self.reinits = reinit, max_reinits, 0
        self._lock = threading.Lock()
        self._stop = False
        self._thread = threading.Thread(target=self._watch, name="fhespear-fence", daemon=True)
        self._thread.start()

    def _k(self, *parts):
        return self.PREFIX + "/".join(str(p) for p in parts)

    def _get(self, key):
        return self.store.get(key).decode() if self.store.check([key]) else None

    def _abort(self):
        with self._lock:
            if self.aborted:
                return
            self.aborted = True
        try:
            self.d.distributed_c10d._abort_process_group()
        except Exception as e:   # reported, never hidden
            self.log(f"fence: rank {self.rank} process-group abort raised {type(e).__name__}: {e}")

    def _watch(self):
        import time
        while not self._stop:
            time.sleep(self.poll_s)
            act = self.active
            if act is None or self.tripped is not None:
                continue
            seq, name, t0 = act
            try:
                msg = self._get(self._k("fail", seq))
            except Exception:
                continue
            limit = self.leg_timeout_s * (2 if self.waiting else 1)
            if msg is None and time.time() - t0 > limit:
                msg = (f"rank {self.rank}: leg {name!r} still running after {limit:.0f} s"
                       + (" (waiting in a collective)" if self.waiting else ""))
                try:
                    self.store.set(self._k("fail", seq), msg)
                except Exception:
                    pass
            if msg is not None and self.active is act:
                self.tripped = msg
                self.log(f"fence: rank {self.rank} leaves leg {name!r}: {msg}")
                self._abort()

    def check(self):
        """PeerFailed when another rank has failed in the running leg."""
        if self.tripped is not None:
            raise PeerFailed(self.tripped)

    def point(self, stage):
        """A stage boundary of the running leg: check(), then the injected failure if one is due here."""
        self.check()
        act = self.active
        if act is not None and (act[1], stage, self.rank) in self.inject:
            raise InjectedFailure(f"injected failure in leg {act[1]!r} at {stage!r} on rank {self.rank}")

    def run(self, name, fn, *a, **k):
        """fn(*a, **k) as leg `name` on every rank -> (result, fault); fault is None when every rank completed
        the leg, else the same dict on every rank."""
        import json
        import time
        if self.aborted:
            return None, {"skipped": f"process group aborted after leg {self.failed_leg!r} failed"}
        with self._lock:
            self.seq += 1
            seq = self.seq
            self.tripped = None
            self.active = (seq, name, time.time())
        res, err = None, None
        try:
            if (name, None, self.rank) in self.inject:
                raise InjectedFailure(f"injected failure at the start of leg {name!r} on rank {self.rank}")
            res = fn(*a, **k)
            self.check()
        except PeerFailed as e:   # this rank's own watcher may have timed the leg out: that is this rank's failure
            err = ("self" if str(e).startswith(f"rank {self.rank}:") else "peer", str(e)[:400])
        except Exception as e:
            msg = f"{type(e).__name__}: {e}"[:400]
            # a collective that errors because a peer failed first (its abort closed the connection) is that
            # failure's consequence: the peer published its error before aborting
            first = None
            try:
                first = self._get(self._k("fail", seq))
            except Exception:
                pass
            if first is not None and not first.startswith(f"rank {self.rank}:") and not isinstance(e, InjectedFailure):
                err = ("peer", f"{first} (here: {msg})"[:400])
                self.tripped = self.tripped or first
            else:
                err = ("self", msg)
                self.log(f"fence: rank {self.rank} leg {name!r} failed: {msg}")
                try:
                    if first is None:
                        self.store.set(self._k("fail", seq), f"rank {self.rank}: {msg}")
                except Exception:
                    pass
            with self._lock:
                self.active = None   # the watcher has nothing left to report for this leg
            self._abort()
        finally:
            with self._lock:
                self.active = None
        if err is None and self.tripped is not None:   # a peer failed after this rank's last collective
            err = ("self" if self.tripped.startswith(f"rank {self.rank}:") else "peer", self.tripped)
        self.store.set(self._k("status", seq, self.rank),
                       json.dumps({"ok": err is None, "kind": err[0] if err else None, "error": err[1] if err else None}))
        keys = [self._k("status", seq, r) for r in range(self.world)]
        deadline = time.time() + self.agree_timeout_s
        while not self.store.check(keys) and time.time() < deadline:
            time.sleep(0.02)
        stats = {}
        for r, key in enumerate(keys):
            v = self._get(key)
            if v is not None:
                stats[r] = json.loads(v)
        missing = [r for r in range(self.world) if r not in stats]
        if not missing and all(s["ok"] for s in stats.values()):
            return res, None
        first = self._get(self._k("fail", seq))
        fault = {"error": first or f"ranks {missing} did not report leg {name!r} within {self.agree_timeout_s:.0f} s",
                 "failed_ranks": sorted(r for r, s in stats.items() if s["kind"] == "self"),
                 "abandoned_ranks": sorted(r for r, s in stats.items() if s["kind"] == "peer"),
                 "unresponsive_ranks": missing}
        self.failed_leg = name
        self._abort()   # collectives of the failed leg may be half-issued on some rank
        if self.reinit is not None and not missing and self.reinits_left > 0:
            # every rank reported, so every rank is here: a fresh process group for the next legs
            try:
                self.reinits += 1
                self.reinits_left -= 1
                self.reinit(self.d.PrefixStore(self._k("pg", self.reinits), self.store))
                self.aborted = False
                fault["process_group"] = f"re-created ({self.reinits})"
            except Exception as e:   # reported, never hidden: the later legs are skipped
                fault["process_group"] = f"re-creation failed: {type(e).__name__}: {e}"[:300]
        return res, fault

    def finish(self, timeout_s=600.0):
        """After rank 0 printed its line: every rank leaves together.  An intact process group is destroyed
        (barrier first); an aborted one is left alone.  Returns when the caller may exit."""
        import time
        self._stop = True
        if self.rank == 0:
            self.store.set(self._k("done"), "1")
        else:
            deadline = time.time() + timeout_s
            while not self.store.check([self._k("done")]) and time.time() < deadline:
                time.sleep(0.05)
        if not self.aborted:
            self.d.barrier()
            self.d.destroy_process_group()


class LocalFence:
    """FailureFence at world 1 without a process group: each leg's exception is reported, the next leg runs."""

    def __init__(self, log=None):
        import os
        self.inject = parse_inject(os.environ.get("FHESPEAR_BENCH_INJECT"))
        self.log = log or (lambda m: None)
        self.active = None
        self.aborted = False

    def check(self):
        pass

    def point(self, stage):
        if self.active is not None and (self.active, stage, 0) in self.inject:
            raise InjectedFailure(f"injected failure in leg {self.active!r} at {stage!r} on rank 0")

    def run(self, name, fn, *a, **k):
        self.active = name
        try:
            if (name, None, 0) in self.inject:
                raise InjectedFailure(f"injected failure at the start of leg {name!r} on rank 0")
            return fn(*a, **k), None
        except Exception as e:
            msg = f"{type(e).__name__}: {e}"[:400]
            self.log(f"fence: leg {name!r} failed: {msg}")
            return None, {"error": msg, "failed_ranks": [0], "abandoned_ranks": [], "unresponsive_ranks": []}
        finally:
            self.active = None

    def finish(self, timeout_s=0.0):
        pass


def device_identity(ph, local: int):
    """This rank's device: ordinal, PCI bus id (the HIP runtime's), name -- rank 0 gathers them to show
    that RCCL saw N ranks on N distinct GPUs."""
    import os
    import socket
    ident = {"local_rank": local, "device": local, "host": socket.gethostname(),
             "visible": os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")}
    try:
        ident["pci_bus_id"] = ph.device_pci_bus_id(local)
    except Exception as e:   # reported, never hidden
        ident["pci_bus_id"] = f"unavailable: {e}"[:120]
    return ident


def gather_identities(dist, ident):
    """Every rank's device_identity on every rank (object all-gather)."""
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, ident)
    return out


def owner(p: int, world: int) -> int:
    return p % world


def my_projections(n: int, world: int, rank: int) -> list[int]:
    return [p for p in range(n) if owner(p, world) == rank]


def stage_assignment(world: int, rank: int):
    """For each block stage, the projections this rank computes (round-robin inside the stage)."""
    out = []
    for stage in RWKV_BLOCK_STAGES:
        out.append([name for i, name in enumerate(stage) if i % world == rank])
    return out


def gather_to_root(dist, tensor, world: int, rank: int, root: int = 0):
    """All ranks' `tensor` (same shape) -> list on root (None elsewhere)."""
    import torch
    lst = [torch.empty_like(tensor) for _ in range(world)] if rank == root else None
    dist.gather(tensor, lst, dst=root)
    return lst


def broadcast_from(dist, tensor, src: int):
    dist.broadcast(tensor, src=src)
    return tensor


def int64_sum_is_exact(world: int, moduli) -> bool:
    """A plain int64 sum of `world` residues r_i < q stays exact iff world (max q - 1) < 2^63."""
    return world * (max(int(q) for q in moduli) - 1) < 2 ** 63


def modular_reduce_sum(dist, tensor, moduli_per_row, root: int = 0, group=None):
    """Sum of residues across the ranks of `group` (default: all), reduced mod q_i per limb row on
    the global rank `root` (giant-step sharding, §8e(2)).  RCCL's integer sum is not modular: when
    world (max q - 1) < 2^63 (e.g. <= 15 ranks at 59-bit, <= 7 at 60-bit) one int64 reduce and one
    reduction on the root are exact; otherwise the partials are gathered to the root and added mod q
    one at a time (every intermediate < 2 q < 2^63)."""
    import torch
    world = dist.get_world_size(group)
    q = torch.as_tensor([int(m) for m in moduli_per_row], dtype=torch.int64, device=tensor.device).view(-1, 1)
    me = dist.get_rank()
    if int64_sum_is_exact(world, moduli_per_row):
        dist.reduce(tensor, dst=root, group=group)
        if me == root:
            tensor.view(q.shape[0], -1).remainder_(q)
        return tensor
    parts = [torch.empty_like(tensor) for _ in range(world)] if me == root else None
    dist.gather(tensor, parts, dst=root, group=group)
    if me == root:
        acc = tensor.view(q.shape[0], -1)
        acc.zero_()
        for p in parts:
            acc.add_(p.view(q.shape[0], -1))
            acc.sub_(q * (acc >= q))
    return tensor


# ------------------------------------------------------------------ library stream <-> torch stream
_LIB_STREAMS = {}


def lib_stream(ph, ctx):
    """torch view of the context's HIP stream (every library call is ordered on it)."""
    import torch
    key = id(ctx)
    st = _LIB_STREAMS.get(key)
    if st is None or st[0] is not ctx:
        dev = torch.device("cuda", getattr(ctx, "device", torch.cuda.current_device()))
        st = (ctx, torch.cuda.ExternalStream(ph.context_stream(ctx), device=dev))
        _LIB_STREAMS[key] = st
    return st[1]


def _order(first, then):
    """`then` waits (on the device) for the work enqueued so far on `first`."""
    import torch
    ev = torch.cuda.Event()
    ev.record(first)
    then.wait_event(ev)


def to_buffer(ph, ctx, ct, buf):
    """Ciphertext limbs -> torch buffer (int64 view), ordered by events instead of device-wide
    synchronisation: the library stream waits for torch's pending work on `buf` (the allocation's
    previous use), the copy runs on the library stream, torch's current stream waits for the copy
    before any RCCL / torch op reads `buf`."""
    import torch
    cur, lib = torch.cuda.current_stream(buf.device), lib_stream(ph, ctx)
    _order(cur, lib)
    ph.ciphertext_copy_to_device(ctx, ct, buf.data_ptr(), sync=False)
    _order(lib, cur)


def from_buffer(ph, ctx, buf, ncomp, chain_index, scale):
    """torch buffer -> new ciphertext; the library stream waits for the buffer's producer (e.g. an
    RCCL receive on torch's stream), torch waits for the copy before it may reuse `buf`."""
    import torch
    cur, lib = torch.cuda.current_stream(buf.device), lib_stream(ph, ctx)
    _order(cur, lib)
    ct = ph.ciphertext_from_device(ctx, buf.data_ptr(), ncomp, chain_index, scale, sync=False)
    _order(lib, cur)
    return ct


def broadcast_ciphertext(ph, ctx, ct, src: int, dist, device, group=None):
    """Global rank `src`'s ciphertext (None on the other ranks) -> a ciphertext on every rank of `group`:
    a small header (chain index, size, scale) then the limbs as one int64 buffer (RCCL broadcast over
    xGMI; gloo stages both through host memory).  Returns `ct` itself on src."""
    import torch
    me = dist.get_rank()
    host = dist.get_backend(group) == "gloo"
    hdr = torch.zeros(3, dtype=torch.float64, device="cpu" if host else device)
    if me == src:
        hdr.copy_(torch.tensor([ct.chain_index(), ct.size(), ct.scale()], dtype=torch.float64))
    dist.broadcast(hdr, src=src, group=group)
    ci, ncomp, scale = int(hdr[0].item()), int(hdr[1].item()), float(hdr[2].item())
    buf = torch.empty(ncomp * ctx.limbs(ci) * ctx.N, dtype=torch.int64, device=device)
    if me == src:
        to_buffer(ph, ctx, ct, buf)
    if host:
        h = buf.cpu()
        dist.broadcast(h, src=src, group=group)
        if me != src:
            buf.copy_(h)
    else:
        dist.broadcast(buf, src=src, group=group)
    return ct if me == src else from_buffer(ph, ctx, buf, ncomp, ci, scale)


def broadcast_ciphertexts(ph, ctx, cts, src: int, dist, device, n: int, group=None):
    """`n` ciphertexts of one level and scale (e.g. the G baby steps of an input: north_star "baby steps
    computed once and broadcast") from global rank `src` to every rank of `group`, as one buffer."""
    import torch
    me = dist.get_rank()
    host = dist.get_backend(group) == "gloo"
    hdr = torch.zeros(3, dtype=torch.float64, device="cpu" if host else device)
    if me == src:
        hdr.copy_(torch.tensor([cts[0].chain_index(), cts[0].size(), cts[0].scale()], dtype=torch.float64))
    dist.broadcast(hdr, src=src, group=group)
    ci, ncomp, scale = int(hdr[0].item()), int(hdr[1].item()), float(hdr[2].item())
    w = ncomp * ctx.limbs(ci) * ctx.N
    buf = torch.empty(n * w, dtype=torch.int64, device=device)
    if me == src:
        for k, c in enumerate(cts):
            to_buffer(ph, ctx, c, buf[k * w:(k + 1) * w])
    if host:
        h = buf.cpu()
        dist.broadcast(h, src=src, group=group)
        if me != src:
            buf.copy_(h)
    else:
        dist.broadcast(buf, src=src, group=group)
    if me == src:
        return list(cts)
    return [from_buffer(ph, ctx, buf[k * w:(k + 1) * w], ncomp, ci, scale) for k in range(n)]


def send_ciphertext(ph, ctx, ct, src: int, dst: int, dist, device):
    """Point to point: `ct` on global rank src -> a ciphertext on dst (returned there; None elsewhere,
    `ct` itself when src == dst).  Header then limbs; gloo through host memory."""
    import torch
    me = dist.get_rank()
    if src == dst:
        return ct if me == src else None
    if me not in (src, dst):
        return None
    host = dist.get_backend() == "gloo"
    hdr = torch.zeros(3, dtype=torch.float64, device="cpu" if host else device)
    if me == src:
        hdr.copy_(torch.tensor([ct.chain_index(), ct.size(), ct.scale()], dtype=torch.float64))
        dist.send(hdr, dst=dst)
        buf = torch.empty(ct.size() * ct.coeff_modulus_size() * ctx.N, dtype=torch.int64, device=device)
        to_buffer(ph, ctx, ct, buf)
        dist.send(buf.cpu() if host else buf, dst=dst)
        return None
    dist.recv(hdr, src=src)
    ci, ncomp, scale = int(hdr[0].item()), int(hdr[1].item()), float(hdr[2].item())
    buf = torch.empty(ncomp * ctx.limbs(ci) * ctx.N, dtype=torch.int64, device=device)
    if host:
        h = buf.cpu()
        dist.recv(h, src=src)
        buf.copy_(h)
    else:
        dist.recv(buf, src=src)
    return from_buffer(ph, ctx, buf, ncomp, ci, scale)


def stage_groups(n_proj: int, world: int):
    """Latency mode for one block stage: its n_proj projections -> contiguous, balanced groups of
    ranks (sizes differ by <= 1), each group sharding one projection's giant steps.  None when
    there are fewer ranks than projections (the stage is dealt round-robin instead)."""
    if world < n_proj:
        return None
    base, extra = divmod(world, n_proj)
    out, lo = [], 0
    for i in range(n_proj):
        s = base + (1 if i < extra else 0)
        out.append(list(range(lo, lo + s)))
        lo += s
    return out


# ------------------------------------------------------------------ giant-step sharding (§8e(2))
def giant_groups(B: int, world: int, rank: int) -> list[int]:
    """Contiguous, balanced share of the giant groups 0..B-1 for `rank` (sizes differ by <= 1)."""
    if world > B:
        raise ValueError(f"giant_groups: {world} ranks for {B} giant groups")
    base, extra = divmod(B, world)
    lo = rank * base + min(rank, extra)
    return list(range(lo, lo + base + (1 if rank < extra else 0)))


def bsgs_giant_partial(ph, ctx, baby, pts, G: int, D: int, groups, gk, zero_pts):
    """sum_{g in groups} rot_{gG}( sum_b baby[b] (.) pts[gG + b] ), not rescaled (bg:468-483 for a
    subset of g).  `pts` maps a diagonal index to its plaintext (a list, or a dict holding only this
    rank's diagonals); `zero_pts` = G encodings of 0 at the diagonals' level, which fill the identity
    group fhs_linear_transform requires when g = 0 is not ours and pad a short last group."""
    elts, flat = [1], []
    if groups and groups[0] == 0:
        first, rest = [0], groups[1:]
    else:
        first, rest = [], groups
        flat.extend(zero_pts[:G])
    for g in first + list(rest):
        if g:
            elts.append(ph.get_elt_from_step(g * G, ctx.N))
        for b in range(G):
            k = g * G + b
            flat.append(pts[k] if k < D else zero_pts[b])
    return ph.linear_transform(ctx, baby, flat, G, elts, gk, rescale=False)


def bsgs_giant_sharded(ph, ctx, baby, pts, G: int, B: int, D: int, gk, zero_pts, dist, device="cuda",
                       ranks=None, group=None):
    """One matvec with its giant groups split over `ranks` (global ranks of process group `group`;
    default: every rank), gloo staging through host memory.  Returns the rescaled output ciphertext
    on ranks[0], None elsewhere; limb-identical to ph.bsgs_multiply_accumulate(ctx, baby, pts, G, B,
    D, gk).  `pts` need only hold this rank's diagonals."""
    import torch
    me = dist.get_rank()
    ranks = list(range(dist.get_world_size())) if ranks is None else list(ranks)
    share = giant_groups(B, len(ranks), ranks.index(me))
    part = bsgs_giant_partial(ph, ctx, baby, pts, G, D, share, gk, zero_pts)
    ci, scale, l = part.chain_index(), part.scale(), part.coeff_modulus_size()
    buf = torch.empty(2 * l * ctx.N, dtype=torch.int64, device=device)
    to_buffer(ph, ctx, part, buf)
    rows = [int(q) for q in ctx.primes[:l]] * 2   # [comp][limb] rows, limb t mod q_t
    if dist.get_backend(group) == "gloo":
        h = buf.cpu()
        modular_reduce_sum(dist, h, rows, root=ranks[0], group=group)
        buf.copy_(h)
    else:
        modular_reduce_sum(dist, buf, rows, root=ranks[0], group=group)
    if me != ranks[0]:
        return None
    total = from_buffer(ph, ctx, buf, 2, ci, scale)
    return ph.rescale_to_next(ctx, total)


def linear_transform_sharded(ph, ctx, babies, pts, G: int, elts, gk, rescale: bool, zero_pts, dist, device="cuda",
                             ranks=None, group=None):
    """One fused BSGS linear transform (ph.linear_transform: the bootstrap's CoeffToSlot / SlotToCoeff
    groups) with its giant groups split over `ranks` (global ranks of `group`): each rank sums its share
    of the groups before ModDown (the identity group -- zero plaintexts `zero_pts` when it is another
    rank's -- first, as the kernel expects), the partial ciphertexts are summed mod q_i on ranks[0], which
    rescales when asked.  Every term is an exact residue: limb-identical to the one-GPU transform.  A rank
    beyond the number of groups contributes nothing.  Returns the output on ranks[0], None elsewhere."""
    import torch
    me = dist.get_rank()
    ranks = list(range(dist.get_world_size())) if ranks is None else list(ranks)
    n_groups, idx = len(elts), ranks.index(me)
    active = min(len(ranks), n_groups)
    share = giant_groups(n_groups, active, idx) if idx < active else []
    part = None
    if share:
        flat, es = [], [1]
        if share[0] == 0:
            first, rest = [0], share[1:]
        else:
            first, rest = [], share
            flat.extend(zero_pts[:G])
        for g in first + rest:
            if g:
                es.append(elts[g])
            flat.extend(pts[g * G:(g + 1) * G])
        part = ph.linear_transform(ctx, babies, flat, G, es, gk, rescale=False)
    ci = babies[0].chain_index()
    l = ctx.limbs(ci)
    buf = torch.zeros(2 * l * ctx.N, dtype=torch.int64, device=device)
    if part is not None:
        to_buffer(ph, ctx, part, buf)
    rows = [int(q) for q in ctx.primes[:l]] * 2
    if dist.get_backend(group) == "gloo":
        h = buf.cpu()
        modular_reduce_sum(dist, h, rows, root=ranks[0], group=group)
        buf.copy_(h)
    else:
        modular_reduce_sum(dist, buf, rows, root=ranks[0], group=group)
    if me != ranks[0]:
        return None
    total = from_buffer(ph, ctx, buf, 2, ci, babies[0].scale() * pts[0].scale())
    return ph.rescale_to_next(ctx, total) if rescale else total


# ------------------------------------------------------------------ baby-step sharding (§8e(2))
def baby_steps_share(G: int, world: int, rank: int) -> list[int]:
    """Contiguous, balanced share of the baby steps 0..G-1 for `rank` (baby step 0 is the input)."""
    if world > G:
        raise ValueError(f"baby_steps_share: {world} ranks for {G} baby steps")
    base, extra = divmod(G, world)
    lo = rank * base + min(rank, extra)
    return list(range(lo, lo + base + (1 if rank < extra else 0)))


def baby_sharded_rows(G: int, B: int, D: int, world: int, rank: int) -> list[int]:
    """Diagonal indices rank `rank` needs in baby-step-sharded mode: its baby steps' column of every
    giant group."""
    return [g * G + b for g in range(B) for b in baby_steps_share(G, world, rank) if g * G + b < D]


def _reduce_scatter_mod(dist, parts, sizes, moduli_rows, group, host):
    """parts: [world][kmax][W] int64 (rank r's contribution to every owner's slots); returns this
    rank's [kmax][W] sums reduced mod q per limb row.  RCCL's integer sum is exact for world (max q - 1)
    < 2^63 (<= 15 ranks at 59-bit primes); otherwise (or on gloo, which lacks reduce_scatter) the slices
    are reduced one owner at a time with the modular sum of modular_reduce_sum."""
    import torch
    world, kmax, W = parts.shape
    me = dist.get_rank(group) if group is not None else dist.get_rank()
    q = torch.as_tensor([int(m) for m in moduli_rows], dtype=torch.int64, device=parts.device).view(-1, 1)
    if not host and int64_sum_is_exact(world, moduli_rows):
        out = torch.empty((kmax, W), dtype=torch.int64, device=parts.device)
        dist.reduce_scatter_tensor(out, parts.reshape(-1), group=group)
        out.view(kmax, q.shape[0], -1).remainder_(q)
        return out
    out = None
    for owner in range(world):
        buf = parts[owner].clone()
        root = owner if group is None else dist.get_global_rank(group, owner)
        modular_reduce_sum(dist, buf, list(moduli_rows) * kmax, root=root, group=group)
        if owner == me:
            out = buf
    return out


def _rows_tensor(rows, device):
    import torch
    return torch.as_tensor([int(q) for q in rows], dtype=torch.int64, device=device).view(-1, 1)


def grid_shape(world: int, rb: int):
    """Rank index idx of a world = rb x rg grid -> (baby share i = idx % rb, giant column j = idx // rb)."""
    if rb < 1 or world % rb:
        raise ValueError(f"grid: {world} ranks do not split into {rb} baby shares")
    return rb, world // rb


def grid_rb(R: int) -> int:
    """Baby shares of the grid for a projection sharded over R ranks (BlockRunner shard="grid").  Per-rank
    compute measured alone on one MI355X at cfg2 (HISTORY.md §6, profiles/r03/grid_shard_cfg2_projection.log)
    plus the reduce-scatter's xGMI time at ~64 GB/s per link and direction ((rb - 1)/rb x |column| x 9.4 MB
    per rank, spread over the rb - 1 peers' direct links): at 2-4 ranks the transfer outweighs the baby
    rotations it saves (2x1 4.5 + ~3.3 ms vs 1x2 5.0 ms; 2x2 3.0 + ~1.7 vs 1x4 3.5), at 8 ranks sharding
    all baby steps wins (8x1 1.7 + ~0.8 ms vs 1x8 2.7 ms, 4x2 1.8 + ~0.8)."""
    return R if R >= 8 else 1


def column_shares(n: int, rb: int) -> list[list[int]]:
    """A giant column of n groups split over its rb ranks in ceil(n / rb)-sized contiguous slices (the
    last shorter), so slice r sits at slots [r k, r k + len) of a [rb k] reduce-scatter buffer without
    reordering; every rank gets at least one group when (rb - 1) ceil(n / rb) < n."""
    k = -(-n // rb)
    if (rb - 1) * k >= n:
        raise ValueError(f"grid: a column of {n} giant groups leaves a rank of {rb} without a group")
    return [list(range(r * k, min((r + 1) * k, n))) for r in range(rb)]


def grid_groups(dist, ranks, rb: int):
    """The process groups of the grid's giant columns (the rb ranks that reduce-scatter one column's
    partial inner products).  Every process of the default group must call this with the same
    arguments (torch.distributed.new_group is collective); returns {column: group}."""
    ranks = list(ranks)
    rb, rg = grid_shape(len(ranks), rb)
    return {j: dist.new_group(ranks=ranks[j * rb:(j + 1) * rb]) for j in range(rg)} if rb > 1 else {}


def bsgs_grid_sharded(ph, ctx, ct, pts, G: int, B: int, D: int, gk, zero_diag, dist, rb: int, device="cuda",
                      ranks=None, group=None, col_groups=None, timings=None, sim_grid=None):
    """One matvec over R = rb x rg ranks (latency mode): the B giant groups are split
    into rg contiguous columns (giant_groups) and the G baby steps into rb shares (baby_steps_share).
    Rank (i, j) rotates the input by its baby share (hoisted inside the library), forms the partial
    inner products of column j's groups over that share (ph.bsgs_inner_products), the rb ranks of
    column j reduce-scatter them (int64 RCCL sum + one reduction mod q_i, exact for rb <= 15) so each
    holds the full inner products of its slice of the column, and key-switches and sums only those
    (ph.bsgs_giant_steps: one key switch per group, summed before one ModDown).  The partial outputs
    are summed mod q_i on ranks[0] (modular_reduce_sum), which rescales.  Every term is an exact
    residue, so the result is limb-identical to ph.bsgs_multiply_accumulate on one GPU.
    rb = 1 is giant-step sharding (every rank rotates all G baby steps, no reduce-scatter); rb = R is
    baby-step sharding (one column); in between trades the replicated baby rotations against the
    reduce-scatter volume ((rb - 1) / rb x |column| x 2 l N x 8 bytes per rank).
    `pts` maps a diagonal index to its plaintext and need only hold grid_rows of this rank;
    zero_diag: an encoding of 0 at the diagonals' level and scale (pads the short last group);
    col_groups: grid_groups(dist, ranks, rb) (made here when None -- collective over all ranks);
    timings: optional dict that receives per-phase seconds (device-synchronised; diagnostics);
    sim_grid = (rb, rg) (diagnostics, one process): run rank (0, 0)'s share of that grid alone, the two
    collectives replaced by their local part (the mod-q reduction of this rank's slice, no transfer)."""
    import time
    import torch
    me = dist.get_rank()
    ranks = list(range(dist.get_world_size())) if ranks is None else list(ranks)
    R, idx = len(ranks), ranks.index(me)
    if sim_grid is not None:
        (rb, rg), idx, ranks = sim_grid, 0, [me]
    else:
        rb, rg = grid_shape(R, rb)
    i, j = idx % rb, idx // rb
    host = dist.get_backend(group) == "gloo"
    if col_groups is None and sim_grid is None:
        col_groups = grid_groups(dist, ranks, rb)
    t0 = [time.perf_counter()]

    def mark(name):
        if timings is not None:
            ctx.synchronize()
            torch.cuda.synchronize(device)
            t = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + t - t0[0]
            t0[0] = t
    col = giant_groups(B, rg, j)
    shares = column_shares(len(col), rb)            # positions in col, contiguous: slot = position
    my_groups = [col[x] for x in shares[i]]
    bs = baby_steps_share(G, rb, i)
    baby = [ct if b == 0 else ph.rotate(ctx, ct, b, gk) for b in bs]
    flat = [pts[g * G + b] if g * G + b < D else zero_diag for g in col for b in bs]
    ci, l = ct.chain_index(), ct.coeff_modulus_size()
    scale = ct.scale() * flat[0].scale()
    W = 2 * l * ctx.N
    rows = [int(q) for q in ctx.primes[:l]] * 2
    elts = [ph.get_elt_from_step(g * G, ctx.N) if g else 1 for g in my_groups]
    if rb == 1:   # giant-step sharding: one fused linear transform over this rank's groups
        part = bsgs_giant_partial(ph, ctx, baby, pts, G, D, col, gk, [zero_diag] * G)
        del baby
        mark("baby+inner")
    else:
        kmax = len(shares[0])
        parts = torch.empty((rb * kmax, W), dtype=torch.int64, device=device)
        if rb * kmax > len(col):
            parts[len(col):].zero_()
        cur, lib = torch.cuda.current_stream(parts.device), lib_stream(ph, ctx)
        _order(cur, lib)                             # the buffer's previous users before the library writes
        ph.bsgs_inner_products_to_device(ctx, baby, flat, len(bs), len(col), parts.data_ptr())
        _order(lib, cur)
        del baby
        mark("baby+inner")
        if sim_grid is not None:   # one contribution: only the local mod-q reduction of this rank's slice
            mine = parts[:kmax]
            mine.view(kmax, len(rows), -1).remainder_(_rows_tensor(rows, device))
        elif host:
            mine = _reduce_scatter_mod(dist, parts.view(rb, kmax, W).cpu(), len(shares[i]), rows, col_groups[j],
                                       True).to(device)
        else:
            mine = _reduce_scatter_mod(dist, parts.view(rb, kmax, W), len(shares[i]), rows, col_groups[j], False)
        mark("reduce_scatter")
        _order(cur, lib)
        part = ph.bsgs_giant_steps_from_device(ctx, mine.data_ptr(), len(my_groups), ci, scale, elts, gk)
        _order(lib, cur)                             # torch may reuse `mine` only after the library read it
        del mine, parts
    mark("giant")
    buf = torch.empty(W, dtype=torch.int64, device=device)
    to_buffer(ph, ctx, part, buf)
    if sim_grid is not None:
        buf.view(len(rows), -1).remainder_(_rows_tensor(rows, device))
    elif host:
        h = buf.cpu()
        modular_reduce_sum(dist, h, rows, root=ranks[0], group=group)
        buf.copy_(h)
    else:
        modular_reduce_sum(dist, buf, rows, root=ranks[0], group=group)
    mark("reduce")
    if me != ranks[0]:
        return None
    total = from_buffer(ph, ctx, buf, 2, ci, part.scale())
    out = ph.rescale_to_next(ctx, total)
    mark("rescale")
    return out


def grid_rows(G: int, B: int, D: int, world: int, rb: int, rank: int) -> list[int]:
    """Diagonal indices rank index `rank` of an rb x (world / rb) grid needs: its baby share's column of
    each giant group of its column."""
    rb, rg = grid_shape(world, rb)
    return [g * G + b for g in giant_groups(B, rg, rank // rb) for b in baby_steps_share(G, rb, rank % rb)
            if g * G + b < D]


def bsgs_baby_sharded(ph, ctx, ct, pts, G: int, B: int, D: int, gk, zero_diag, dist, device="cuda",
                      ranks=None, group=None, col_groups=None, timings=None):
    """Baby-step sharding: bsgs_grid_sharded with rb = R (one giant column)."""
    R = dist.get_world_size() if ranks is None else len(ranks)
    return bsgs_grid_sharded(ph, ctx, ct, pts, G, B, D, gk, zero_diag, dist, R, device, ranks, group,
                             col_groups if col_groups is not None else {0: group}, timings)
