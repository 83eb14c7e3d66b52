"""Data parallelism: one process per GPU, gradient all-reduce over RCCL (xGMI).

Replaces the reference's single-process <=4-replica scheme
(/root/reference/utils/training_utils.py:131-303, train.py:67-78): there, every
parameter's gradient is copied to cuda:0, averaged, stepped once, and every
parameter is copied back, with nothing overlapped.  Here:

  * each rank runs the identical Seq2Seq on its own batches; rank r of n takes
    batches r, r+n, r+2n, ... of one common seeded order, and leftover batches
    are dropped (the reference's rule, training_utils.py:160,180-184);
  * the loss gradient is pre-scaled by 1/n, so a SUM all-reduce of the flat
    gradient arena gives the mean gradient of the n*B global batch (what the
    reference's averaging computes);
  * the arena is laid out in reverse backward order (engine.py), so after each
    layer's backward a contiguous prefix of the arena is final; buckets of
    >= bucket_bytes are all-reduced asynchronously as soon as they are complete,
    on RCCL's own stream, overlapping the remaining backward;
  * clip + Adam then run replicated on every rank on identical reduced grads.

NSTL_DP=zero1 (ShardComm + utils.optim.FusedAdam.shard): after
backward the gradient arena is reduce-scattered (f32), each rank clips with the
global norm (one all-reduce of 1024 partial sums) and runs Adam on its 1/n
shard, and the updated compute-dtype parameters are all-gathered.  Per step and
rank that moves (n-1)/n of 4 + 2 bytes per parameter instead of an
all-reduce's 2 * 4, and the optimizer's 30 B/param of HBM traffic drops to 1/n.
The f32 master weights and Adam moments outside a rank's shard go stale until
consolidate() (checkpoints).

Default mode (NSTL_DP=zero1_push, ShardPusher): the same sharded step, but the
reduce-scatter leaves the critical path without any collective kernel in
backward: each final bucket's slices are pushed into their owners' IPC-mapped
receive slots by the copy engines (no CU taken from the step's persistent
grids; measured on one GPU with the same 824 MB of copy-engine traffic per step
as 8 ranks push: +2.1 % step time, tools/copy_interference.py), and each owner
sums its shard in the pass that computes the clip norm's partials.  Setup that
fails on any rank falls back to zero1 on every rank.

NSTL_DP=zero1_overlap (GradShardReducer) moves the reduction into backward: as
soon as a bucket of the arena is final it is reduced (SUM) onto the rank whose
shard holds it, on RCCL's stream, so the reduce-scatter leaves the critical
path; buckets never straddle a shard boundary, and the post-backward step skips
its reduce-scatter.  A collective kernel resident during backward holds CUs the
step's persistent grids would otherwise use: run the compute stream on a CU
mask that cedes them evenly over the XCD shader engines (NSTL_CEDE_CUS, one CU per (XCD, SE) at 32;
nstl_stream_cus then sizes the GEMM / attention grids to the CUs left;
tools/cu_mask_bench.py measures what that costs).
"""
import os

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 64 << 20


class PushTimeout(RuntimeError):
    """A copy-engine copy of the zero1_push exchange did not complete in time."""


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK).
    Returns (rank, world, local_rank); (0, 1, 0) when not launched distributed."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    # NSTL_DIST_BACKEND=gloo: rehearsal of the multi-rank path with several ranks on
    # the GPUs there are (rank -> GPU local % count); gloo carries the collectives
    backend = backend or os.environ.get("NSTL_DIST_BACKEND") or None
    if backend == "gloo" and torch.cuda.is_available():
        local = local % torch.cuda.device_count()
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


_CEDED = {}


_ACTIVE_CEDE = {}  # device index -> k of the ceded compute stream (cede_cus)


def _masked_stream(k, device):
    """A new stream of `device` whose CU mask leaves out mask bits 0 .. k-1."""
    import ctypes
    from . import _hip
    fn = ctypes.CDLL(_hip.LIB_PATH).hipExtStreamCreateWithCUMask
    fn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
    n = torch.cuda.get_device_properties(device).multi_processor_count
    words = (n + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for c in range(k, n):
        mask[c // 32] |= 1 << (c % 32)
    with torch.cuda.device(device):
        st = ctypes.c_void_p()
        if fn(ctypes.byref(st), words, mask) != 0:
            raise RuntimeError("hipExtStreamCreateWithCUMask failed")
    return torch.cuda.ExternalStream(st.value, device=device)


def side_stream(device):
    """A second compute stream for `device` (the engine's weight-gradient stream,
    the optimizer's update stream): with the CU mask of the ceded compute stream
    when cede_cus is active there, so persistent grids launched on it size
    themselves to the same CUs (nstl_stream_cus) and leave the ceded ones to the
    collectives; otherwise a plain stream."""
    k = _ACTIVE_CEDE.get(torch.device(device).index, 0)
    return _masked_stream(k, device) if k > 0 else torch.cuda.Stream(device)


def cede_cus(k, device):
    """Make the current stream of `device` a stream whose CU mask leaves out mask
    bits 0 .. k-1 -- bit i is a CU of XCD i % 8, shader engine (i / 8) % 4
    (tools/micro/cu_probe.hip), so k a multiple of 32 cedes k / 32 CUs of every
    (XCD, SE) pair, the only balanced choices -- for the collective kernels that
    run during backward (NSTL_DP=zero1_overlap).  Returns the stream (kept alive
    here); k <= 0 leaves the current stream."""
    if k <= 0:
        return torch.cuda.current_stream(device)
    key = (torch.device(device).index, k)
    if key not in _CEDED:
        _CEDED[key] = _masked_stream(k, device)
    s = _CEDED[key]
    torch.cuda.set_stream(s)
    _ACTIVE_CEDE[key[0]] = k
    return s


def shard_batch_indices(num_batches, rank, world):
    """Batch indices rank `rank` consumes in one epoch: r, r+n, ... over the
    steps_per_epoch = num_batches // world full rounds (leftovers dropped)."""
    steps = num_batches // world
    return [s * world + rank for s in range(steps)]


class GradAllReducer:
    """Bucketed asynchronous SUM all-reduce over a flat gradient arena.

    ``min_world``: below this many ranks nothing is launched (an all-reduce
    over one rank is the identity); 1 makes a single-rank group run the real
    collectives (tests and tools/rccl_probe.py: RCCL kernels resident beside a
    backward on one GPU)."""

    def __init__(self, grads, group=None, bucket_bytes=DEFAULT_BUCKET_BYTES, min_world=2):
        self.g = grads
        self.group = group
        self.bucket = max(1, bucket_bytes // grads.element_size())
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.active = dist.is_initialized() and self.world >= min_world
        # a finish() completed and no optimizer step has consumed it yet: the arena
        # holds reduced gradients (the step must not reduce them again)
        self.completed = False
        self.reset()

    def reset(self):
        self.sent = 0
        self.works = []

    def begin(self, fresh):
        """Start of a backward.  Drops what an aborted backward left (its buckets
        are waited for, its progress reset).  ``fresh`` False (the backward adds to
        the arena: gradient accumulation) after a completed in-backward reduction
        would count the other ranks' earlier micro-batches twice, so it raises."""
        if not self.active:
            return
        for w in self.works:
            w.wait()
        self.reset()
        if not fresh and self.completed:
            raise RuntimeError("gradient accumulation over several backwards per step is not supported by the "
                               "in-backward reduction (NSTL_DP=%s): the first backward's gradients are already "
                               "reduced; use NSTL_DP=zero1" % self.mode)
        self.completed = False

    def consume(self):
        """Whether the arena holds this step's reduced gradients (a finish()
        completed since the last call); resets the flag."""
        done, self.completed = self.completed, False
        return done

    mode = "allreduce"

    def ready(self, upto):
        """Arena prefix [0, upto) is final: launch buckets of the unsent part."""
        if not self.active:
            return
        while upto - self.sent >= self.bucket:
            self._launch(self.sent, self.sent + self.bucket)

    def _launch(self, lo, hi):
        self.works.append(dist.all_reduce(self.g[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self.sent = hi

    def finish(self):
        """Reduce the tail and make the current stream wait for every bucket."""
        if not self.active:
            return
        if self.sent < self.g.numel():
            self._launch(self.sent, self.g.numel())
        for w in self.works:
            w.wait()
        self.reset()
        self.completed = True


class GradShardReducer(GradAllReducer):
    """ZeRO-1 with the reduction overlapped with backward: bucketed SUM reduce of
    each final arena prefix onto the owning rank of `comm` (ShardComm), cut at
    shard boundaries; [comm.numel, end) -- the replicated tail -- is left to
    zero1_step.  After finish(), rank r's arena [comm.lo, comm.hi) holds the
    summed gradients (what the reduce-scatter would have written)."""

    mode = "zero1_overlap"

    def __init__(self, grads, comm, bucket_bytes=DEFAULT_BUCKET_BYTES, min_world=2):
        self.comm = comm
        super().__init__(grads, comm.group, bucket_bytes, min_world)

    def ready(self, upto):
        if not self.active:
            return
        upto = min(upto, self.comm.numel)
        while self.sent < upto:
            owner = self.sent // self.comm.shard
            end = min((owner + 1) * self.comm.shard, self.sent + self.bucket)
            if end > upto:
                return
            self._reduce(self.sent, end, owner)

    def _reduce(self, lo, hi, owner):
        dst = dist.get_global_rank(self.group, owner) if self.group is not None else owner
        self.works.append(dist.reduce(self.g[lo:hi], dst=dst, op=dist.ReduceOp.SUM, group=self.group,
                                      async_op=True))
        self.sent = hi

    def finish(self):
        if not self.active:
            return
        while self.sent < self.comm.numel:
            owner = self.sent // self.comm.shard
            self._reduce(self.sent, min((owner + 1) * self.comm.shard, self.sent + self.bucket), owner)
        for w in self.works:
            w.wait()
        self.reset()
        self.completed = True


def push_streams():
    """NSTL_PUSH_STREAMS: copy streams of the copy-engine exchange.  Default 1:
    on one GPU with an 8-rank push volume the step pays +2.85 % with one stream,
    +3.8 / +5.6 / +8.5 % with 2 / 3 / 7 (profiles/r5_push_streams.txt); one
    engine moves the 824 MB in ~14 ms at ~60 GB/s, inside the backward."""
    return int(os.environ.get("NSTL_PUSH_STREAMS", "1"))


class _DeviceTransport:
    """The receive buffers of a ShardPusher in device memory, shared between the
    ranks' processes through HIP IPC handles (nstl_ipc_*); pushes are copy-engine
    copies (nstl_copy_engine: hipMemcpyDeviceToDeviceNoCU, no kernel) on
    NSTL_PUSH_STREAMS side streams (owner r on stream r mod n).  xGMI is point to
    point, so more streams put the copies to different peers on different links
    and copy engines at once; on one GPU, though, concurrent copy engines cost the
    step more than their bytes, hence the measured default."""

    def __init__(self, grads, comm, n_slots):
        from . import _hip as K
        self.K = K
        self.shard = comm.shard
        self.gmap = {}
        self._opened = []
        self.sides, self.gsides, self._pool, self.recv = {}, {}, [], None
        # a local failure is recorded, not raised, until every rank has taken the
        # same collectives (ShardPusher raises it afterwards; create() agrees):
        # a rank whose receive buffer or streams cannot be made (e.g. out of
        # memory: (world - 1) f32 shards, ~0.8 GB at 8 ranks) still takes the
        # handle exchange, with no handle of its own
        self.error = None
        try:
            self.recv = torch.empty(max(1, n_slots) * comm.shard, dtype=torch.float32, device=grads.device)
            n = max(1, min(push_streams(), comm.world - 1))
            pool = [torch.cuda.Stream(grads.device) for _ in range(n)]
            self.sides = {r: pool[r % n] for r in range(comm.world) if r != comm.rank}
            # the weight all-gather runs alone between the optimizer and the next
            # forward (no compute beside it to disturb): one stream per peer, so the
            # seven copies travel seven links at once
            self.gsides = {r: torch.cuda.Stream(grads.device) for r in range(comm.world) if r != comm.rank}
            self._pool = pool + list(self.gsides.values())
        except Exception as e:  # noqa: BLE001
            self.error = e
        self.device = grads.device
        self.peer = self._exchange(self.recv, comm)

    def _exchange(self, t, comm):
        """IPC handle of t to every rank, every peer's t mapped here (a collective;
        failures recorded in self.error).  Before a peer on another device is
        mapped, hipDeviceCanAccessPeer must allow this device to reach it (the
        copy engines write over xGMI into the mapping)."""
        mine = None
        if t is not None:
            try:
                mine = self.K.ipc_handle(t) + (t.device.index,)
            except Exception as e:  # noqa: BLE001
                mine, self.error = None, self.error or e
        allh = [None] * comm.world
        dist.all_gather_object(allh, mine, group=comm.group)
        peers = {}
        here = self.device.index
        for r, hh in enumerate(allh):
            if r == comm.rank:
                continue
            if hh is None:
                self.error = self.error or RuntimeError("rank %d has no IPC handle" % r)
                continue
            if hh[2] != here and not torch.cuda.can_device_access_peer(here, hh[2]):
                self.error = self.error or RuntimeError("hipDeviceCanAccessPeer(%d, %d) = 0: rank %d's memory is "
                                                        "not reachable from this device" % (here, hh[2], r))
                continue
            try:
                base = self.K.ipc_open(hh[0])
            except Exception as e:  # noqa: BLE001
                self.error = self.error or e
                continue
            self._opened.append(base)
            peers[r] = base + hh[1]
        return peers

    def push(self, owner, slot, off, src):
        """src (a contiguous f32 slice of the arena) -> owner's receive slot `slot`
        at element offset `off`; ordered after the work queued on the current
        stream so far."""
        if off < 0 or off + src.numel() > self.shard:
            raise ValueError("push of %d elements at %d leaves the %d-element slot" % (src.numel(), off, self.shard))
        side = self.sides[owner]
        side.wait_stream(torch.cuda.current_stream(src.device))
        dst = self.peer[owner] + (slot * self.shard + off) * 4
        self.K.copy_engine(dst, src, src.numel() * 4, stream=side.cuda_stream)

    def mark(self):
        """[(event, peers)]: an event recorded on every copy stream now, with the
        peers whose copies that stream carries (pending() names them)."""
        out = []
        for st in self._pool:
            ev = torch.cuda.Event()
            ev.record(st)
            out.append((ev, sorted(r for r, s in list(self.sides.items()) + list(self.gsides.items()) if s is st)))
        return out

    @staticmethod
    def pending(marks):
        """The peers whose copies behind `marks` have not completed (a host-side
        query: nothing waits)."""
        return sorted({r for ev, peers in marks if not ev.query() for r in peers})

    def map(self, t, comm):
        """Every peer's copy of t, IPC-mapped (a collective on first use of t)."""
        key = (t.data_ptr(), t.numel(), t.dtype)
        if key not in self.gmap:
            self.gmap[key] = self._exchange(t, comm)
        return self.gmap[key]

    def gather(self, t, lo, hi, comm):
        """The all-gather of t (a device tensor every rank holds at the same shape)
        by the copy engines: this rank's elements [lo, hi) (the updated shard) go
        to the same offsets of every peer's t, one stream per peer (gsides).  Each
        peer's t is IPC-mapped once (t must keep its storage: the engine's arenas
        do)."""
        peers = self.map(t, comm)
        esz = t.element_size()
        cur = torch.cuda.current_stream(t.device)
        for r, base in peers.items():
            side = self.gsides[r]
            side.wait_stream(cur)
            self.K.copy_engine(base + lo * esz, t[lo:hi], (hi - lo) * esz, stream=side.cuda_stream)

    def flush(self):
        cur = torch.cuda.current_stream(self.device)
        for side in self._pool:
            cur.wait_stream(side)

    def sync(self, group):
        """Every rank's pushes into every receive buffer have landed."""
        if dist.get_backend(group) == "nccl":
            # stream-ordered: each rank's all-reduce starts after its own pushes
            # (flush) and ends after every rank's has started
            dist.all_reduce(torch.zeros(1, device=self.device), group=group)
        else:
            torch.cuda.current_stream(self.device).synchronize()
            dist.barrier(group=group)

    def slots(self, n_slots):
        return self.recv[:n_slots * self.shard].view(n_slots, self.shard) if n_slots else self.recv[:0].view(0, 0)

    def close(self):
        for base in self._opened:
            self.K.ipc_close(base)
        self._opened = []


class _HostTransport:
    """The same over host memory (CPU tests with gloo): each rank's receive
    buffer is a shared file under /dev/shm that every rank maps."""

    def __init__(self, grads, comm, n_slots):
        import uuid
        tag = [uuid.uuid4().hex if comm.rank == 0 else None]
        dist.broadcast_object_list(tag, src=dist.get_global_rank(comm.group, 0) if comm.group is not None else 0,
                                   group=comm.group)
        self.shard = comm.shard
        self.error = None
        n = max(1, n_slots) * comm.shard
        self.paths = {r: "/dev/shm/nstl_push_%s_%d" % (tag[0], r) for r in range(comm.world)}
        self.recv, self.peer = None, {}
        # failures are recorded, and every rank still takes both barriers
        # (create() agrees on the outcome afterwards)
        try:
            self.recv = torch.from_file(self.paths[comm.rank], shared=True, size=n, dtype=torch.float32)
        except Exception as e:  # noqa: BLE001
            self.error = e
        dist.barrier(group=comm.group)
        for r, p in self.paths.items():
            if r == comm.rank:
                continue
            try:
                self.peer[r] = torch.from_file(p, shared=True, size=n, dtype=torch.float32)
            except Exception as e:  # noqa: BLE001
                self.error = self.error or e
        dist.barrier(group=comm.group)
        if self.recv is not None:
            os.unlink(self.paths[comm.rank])  # mapped by every rank: the memory stays until they exit

    def push(self, owner, slot, off, src):
        if off < 0 or off + src.numel() > self.shard:
            raise ValueError("push of %d elements at %d leaves the %d-element slot" % (src.numel(), off, self.shard))
        o = slot * self.shard + off
        self.peer[owner][o:o + src.numel()].copy_(src)

    def mark(self):
        return []  # the copies above are synchronous

    @staticmethod
    def pending(marks):
        return []

    def flush(self):
        pass

    def sync(self, group):
        dist.barrier(group=group)

    def slots(self, n_slots):
        return self.recv[:n_slots * self.shard].view(n_slots, self.shard) if n_slots else self.recv[:0].view(0, 0)

    def close(self):
        pass


class ShardPusher(GradAllReducer):
    """ZeRO-1 with the reduction moved onto the copy engines (NSTL_DP=zero1_push).

    As soon as a bucket of the gradient arena is final (backward's reverse-order
    prefix, engine.py), each slice of it that another rank's shard holds is
    pushed into that owner's receive buffer -- a slot per sending rank, mapped
    from the owner's memory through an IPC handle -- by a device-to-device copy
    on the copy engines.  No collective kernel runs during backward, so the
    step's one-tile-per-CU persistent grids keep every CU (the CU-mask route,
    zero1_overlap, cost +33 %: DESIGN.md section 5).  After backward one tiny
    collective orders every push before the optimizer, and the owner forms its
    shard's gradient as own + the slots in rank order in the pass that already
    computes the clip norm's sums of squares (nstl_shard_sum), then runs the
    sharded Adam and the bf16 all-gather as zero1 does.

    Pushes overwrite the slots, so a second backward before the step (gradient
    accumulation) simply pushes the accumulated slices again; a step after a
    backward that did not finish falls back to the reduce-scatter (consume())."""

    mode = "zero1_push"

    def __init__(self, grads, comm, bucket_bytes=DEFAULT_BUCKET_BYTES, min_world=2, gather=()):
        self.comm = comm
        super().__init__(grads, comm.group, bucket_bytes, min_world)
        self.n_slots = comm.world - 1
        self.transport = None
        if self.active:
            self.transport = (_DeviceTransport if grads.is_cuda else _HostTransport)(grads, comm, self.n_slots)
            if isinstance(self.transport, _DeviceTransport):
                # the all-gather's targets (the weight arena) mapped now, so that a
                # mapping failure falls back to zero1 on every rank (create) rather
                # than surfacing in the first optimizer step
                for t in gather:
                    self.transport.map(t, comm)

    def setup_error(self):
        """A local failure of the transport's setup (every rank took the same
        collectives regardless), or None."""
        return getattr(self.transport, "error", None)

    def _self_test(self, n=256, timeout_s=None):
        """Every rank pushes a marker into its slot of every peer's receive buffer
        over the real path (IPC mapping + copy engine between devices), then checks
        the markers its peers pushed.  Raises on a missing or wrong marker, so that
        create() falls back to zero1 on every rank instead of the first step
        training on bad sums.

        The copies are watched from the host before anything is chained behind
        them: events recorded on the copy streams are polled against the deadline
        (NSTL_PUSH_TIMEOUT_S, 60 s), and only once they have completed does the
        compute stream join the copy streams and the ranks sync.  A copy that has
        not landed by then raises PushTimeout naming the peers it was for: a copy
        queue that does not drain cannot be trusted by this process, so create()
        does not fall back but lets it end the process (non-zero exit)."""
        import time
        if timeout_s is None:
            timeout_s = float(os.environ.get("NSTL_PUSH_TIMEOUT_S", "60"))
        n = min(n, self.comm.shard)
        g = self.g
        src = torch.full((n,), float(self.comm.rank + 1), dtype=torch.float32, device=g.device)
        for owner in range(self.comm.world):
            if owner != self.comm.rank:
                self.transport.push(owner, self.slot(self.comm.rank, owner), 0, src)
        marks = self.transport.mark()
        t0 = time.monotonic()
        while True:
            stuck = self.transport.pending(marks)
            if not stuck:
                break
            if time.monotonic() - t0 > timeout_s:
                raise PushTimeout("zero1_push self-test on rank %d: copy-engine copies to rank(s) %s not landed "
                                  "after %.0f s" % (self.comm.rank, stuck, timeout_s))
            time.sleep(0.001)
        self.transport.flush()
        self.transport.sync(self.group)
        slots = self.transport.slots(self.n_slots)
        for k in range(self.n_slots):
            sender = k if k < self.comm.rank else k + 1
            got = slots[k, :n]
            if not bool(torch.all(got == float(sender + 1))):
                raise RuntimeError("zero1_push self-test: slot %d (from rank %d) holds %s, expected %d"
                                   % (k, sender, got[:4].tolist(), sender + 1))

    @classmethod
    def create(cls, grads, comm, **kw):
        """A ShardPusher, or None on EVERY rank when any rank could not map its
        peers' receive buffers (IPC unavailable) or its self-test markers came out
        wrong: the ranks agree, so they all take the same collectives afterwards
        (the caller falls back to zero1).  A copy that never lands raises
        PushTimeout instead (see _self_test)."""
        dev = grads.device if grads.is_cuda else "cpu"

        def agree(err):
            ok = torch.tensor([0.0 if err is not None else 1.0], device=dev)
            dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=comm.group)
            return ok.item() >= 1.0

        def fallback(red, err, what):
            if red is not None:
                red.close()
            import sys
            print("NSTL_DP=zero1_push: %s on some rank (%s); falling back to zero1"
                  % (what, err or "another rank failed"), file=sys.stderr)

        err, red = None, None
        try:
            red = cls(grads, comm, **kw)
            err = red.setup_error()
        except Exception as e:  # noqa: BLE001 -- any setup failure: agree on the fallback
            err = e
        if not agree(err):
            fallback(red, err, "receive buffers not mapped")
            return None
        if red.active:
            # the mapped path exercised once (collectives: every rank gets here)
            try:
                red._self_test()
            except PushTimeout:
                raise
            except Exception as e:  # noqa: BLE001
                err = e
            if not agree(err):
                fallback(red, err, "copy-engine self-test failed")
                return None
        return red

    def slot(self, src_rank, owner):
        """Slot of rank src_rank's contribution in owner's receive buffer."""
        return src_rank if src_rank < owner else src_rank - 1

    def begin(self, fresh):
        # no accumulation check: pushes overwrite the slots (see the class doc).
        # Copies an aborted backward left in flight still read the arena the new
        # backward is about to overwrite: the compute stream waits for them first.
        if not self.active:
            return
        self.transport.flush()
        self.reset()
        self.completed = False

    # the first step's pushed shard sums are checked against RCCL's reduce-scatter
    # of the same arena (NSTL_PUSH_VERIFY=0: not)
    verify_pending = os.environ.get("NSTL_PUSH_VERIFY", "1") != "0"
    failed = False
    check = None

    def verify(self, g_full, g_shard, partial, sumsq_fn, rtol=1e-4):
        """g_shard (own slice + the pushed slots, nstl_shard_sum) against the
        reduce-scatter of the same gradient arena, once (the first step): the
        copies cross devices only on a multi-GPU node, so this is where per-step
        ordering of pushes, sync and owner reads is checked on the hardware.
        The sums add the same f32 terms in another order, so they agree to
        rounding (|diff| <= rtol * max|sum|); a lost or stale slice is off by a
        whole contribution.  The ranks agree on the outcome; on a mismatch this
        step continues with the reduce-scatter's shard (and partial sums of
        squares) and self.failed is set: the step's caller then runs zero1.
        Returns whether the pushed sums were right (on every rank)."""
        self.verify_pending = False
        ref = torch.empty_like(g_shard)
        self.comm.reduce_scatter(g_full[:self.comm.numel], ref)
        diff = float((g_shard - ref).abs().max())
        scale = float(ref.abs().max())
        ok_here = diff <= rtol * scale
        flag = torch.tensor([1.0 if ok_here else 0.0], device=g_shard.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=self.group)
        ok = flag.item() >= 1.0
        self.check = {"max_abs_diff": diff, "max_abs": scale, "rtol": rtol, "ok": ok,
                      "what": "first step: pushed shard sums vs reduce-scatter of the same arena"}
        if not ok:
            import sys
            print("NSTL_DP=zero1_push: pushed shard sums differ from the reduce-scatter (rank %d: max |diff| %.3g of "
                  "max %.3g); this step uses the reduce-scatter, later steps run zero1" % (self.comm.rank, diff, scale),
                  file=sys.stderr)
            g_shard.copy_(ref)
            sumsq_fn(g_shard, partial)
            self.failed = True
        return ok

    def ready(self, upto):
        if not self.active:
            return
        upto = min(upto, self.comm.numel)
        while self.sent < upto:
            owner = self.sent // self.comm.shard
            end = min((owner + 1) * self.comm.shard, self.sent + self.bucket)
            if end > upto:
                return
            self._push(self.sent, end, owner)

    def _push(self, lo, hi, owner):
        if owner != self.comm.rank:
            self.transport.push(owner, self.slot(self.comm.rank, owner), lo - owner * self.comm.shard, self.g[lo:hi])
        self.sent = hi

    def finish(self):
        if not self.active:
            return
        while self.sent < self.comm.numel:
            owner = self.sent // self.comm.shard
            self._push(self.sent, min((owner + 1) * self.comm.shard, self.sent + self.bucket), owner)
        self.transport.flush()
        self.transport.sync(self.group)
        self.reset()
        self.completed = True

    def slots(self):
        """This rank's receive slots [world - 1][shard]: slot k = rank k (k < rank)
        or k + 1."""
        return self.transport.slots(self.n_slots)

    def all_gather(self, tensors):
        """After the sharded Adam: every tensor's shard [lo, hi) to every peer
        (copy engines over IPC mappings of the peers' tensors, as the gradient
        pushes), then one stream-ordered sync, so the next forward on every rank
        reads whole weights.  The host transport (CPU tests) all-gathers with
        the collective."""
        if not isinstance(self.transport, _DeviceTransport):
            for t in tensors:
                self.comm.all_gather(t[:self.comm.numel])
            return
        for t in tensors:
            self.transport.gather(t, self.comm.lo, self.comm.hi, self.comm)
        self.transport.flush()
        self.transport.sync(self.group)

    def close(self):
        if self.transport is not None:
            self.transport.close()


class ShardComm:
    """Equal contiguous shards of a flat arena over the ranks of `group`:
    reduce-scatter / all-gather of the arena (torch's tensor collectives, the
    same calls on RCCL and on the gloo backend of the CPU tests)."""

    def __init__(self, numel, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if numel % (self.world * 64):
            raise ValueError("arena of %d elements does not split into %d 64-aligned shards" % (numel, self.world))
        self.numel = numel
        self.shard = numel // self.world
        self.lo = self.rank * self.shard
        self.hi = self.lo + self.shard

    def reduce_scatter(self, full, out):
        """out (this rank's shard) = sum over ranks of full[lo:hi]."""
        dist.reduce_scatter_tensor(out, full, op=dist.ReduceOp.SUM, group=self.group)

    def all_gather(self, full):
        """full[every shard] = the owning rank's full[lo:hi] (in place)."""
        dist.all_gather_into_tensor(full, full[self.lo:self.hi].clone(), group=self.group)


def zero1_step(comm, g_full, g_shard, partial, sumsq_fn, adam_fn, gather, tail=None, reduced=False, sum_fn=None,
               gather_fn=None):
    """One sharded clip + Adam step (the FusedAdam kernels passed in as callables,
    so the orchestration is testable on CPU): reduce-scatter the gradients of
    the shardable region [0, comm.numel) (``reduced``: GradShardReducer already
    summed this rank's shard in place during backward; ``sum_fn``: ShardPusher's
    slots hold the other ranks' slices, and sum_fn(g_shard, partial) forms the
    shard and its sums of squares in one pass), sum of squares of this shard,
    all-reduce of the partial sums; `tail` = (lo, hi), a small replicated region
    (the f32 vectors), is all-reduced whole, its squares added once and updated
    on every rank; Adam on this shard (+ tail), then all-gather each tensor of
    `gather` over the shardable region (``gather_fn(tensors)``: ShardPusher's
    copy-engine all-gather instead of the collective)."""
    if sum_fn is not None:
        sum_fn(g_shard, partial)
    else:
        if reduced:
            g_shard.copy_(g_full[comm.lo:comm.hi])
        else:
            comm.reduce_scatter(g_full[:comm.numel], g_shard)
        sumsq_fn(g_shard, partial)
    dist.all_reduce(partial, op=dist.ReduceOp.SUM, group=comm.group)
    if tail is not None and tail[1] > tail[0]:
        lo, hi = tail
        gt = g_full[lo:hi]
        dist.all_reduce(gt, op=dist.ReduceOp.SUM, group=comm.group)
        part_t = torch.zeros_like(partial)
        sumsq_fn(gt, part_t)
        partial += part_t
        adam_fn(lo, hi - lo, gt, partial)
    adam_fn(comm.lo, comm.shard, g_shard, partial)
    if gather_fn is not None:
        gather_fn(gather)
        return
    for t in gather:
        comm.all_gather(t[:comm.numel])
