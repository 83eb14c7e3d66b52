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
"""
import os

import torch
import torch.distributed as dist

DEFAULT_BUCKET_BYTES = 64 << 20


def init_from_env(backend=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK).
    Returns (rank, world, local_rank); (0, 1, 0) when not launched distributed."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world <= 1:
        return 0, 1, 0
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    if not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def shard_batch_indices(num_batches, rank, world):
    """Batch indices rank `rank` consumes in one epoch: r, r+n, ... over the
    steps_per_epoch = num_batches // world full rounds (leftovers dropped)."""
    steps = num_batches // world
    return [s * world + rank for s in range(steps)]


class GradAllReducer:
    """Bucketed asynchronous SUM all-reduce over a flat gradient arena."""

    def __init__(self, grads, group=None, bucket_bytes=DEFAULT_BUCKET_BYTES):
        self.g = grads
        self.group = group
        self.bucket = max(1, bucket_bytes // grads.element_size())
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.reset()

    def reset(self):
        self.sent = 0
        self.works = []

    def ready(self, upto):
        """Arena prefix [0, upto) is final: launch buckets of the unsent part."""
        if self.world == 1:
            return
        while upto - self.sent >= self.bucket:
            self._launch(self.sent, self.sent + self.bucket)

    def _launch(self, lo, hi):
        self.works.append(dist.all_reduce(self.g[lo:hi], op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        self.sent = hi

    def finish(self):
        """Reduce the tail and make the current stream wait for every bucket."""
        if self.world == 1:
            return
        if self.sent < self.g.numel():
            self._launch(self.sent, self.g.numel())
        for w in self.works:
            w.wait()
        self.reset()
