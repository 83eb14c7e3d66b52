"""Drop-in for utils/training_utils.py (train_one_epoch, train_one_epoch_multi_gpu
and helpers), same signatures, return values, printed lines and plots.

Differences in mechanism, not in meaning:
  * the step is zero_grad -> fused forward/loss -> backward -> one fused
    clip(``clip``)+Adam launch (``FusedAdam.step(max_norm=clip)``); the global
    norm is computed on the device (the reference syncs 344 ``.item()`` per step,
    training_utils.py:349-357).  A plain torch optimizer also works (the
    reference's calculate_gradient_norm / clip_grad_norm_ / step sequence is used).
  * bf16 compute has fp32's exponent range, so no loss scaling is needed: a
    GradScaler passed with ``use_amp=True`` is accepted (as the reference demands,
    :38-39) and left unused.
  * per-step logging reads the loss/norm of step i after step i+1 has been
    queued, so the host never idles the GPU (printed values are the same).
  * multi-GPU is one process per GPU (torch.distributed, RCCL): each rank passes
    its own model; gradients are all-reduced in buckets during backward
    (parallel.GradAllReducer).  The reference's single-process list of replicas
    (training_utils.py:131-303) is also accepted: gradients are averaged into
    models[0]'s arena and parameters copied back, as it does.
"""
import math
import os
import time

import torch
import torch.distributed as dist
import torch.nn as nn

from .optim import FusedAdam


# ---------------------------------------------------------------------------------------------
def _dist():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _engine_of(model):
    return getattr(model, "_engine", None)


def _step_fused(model, optimizer, clip):
    """clip + step; returns the pre-clip global norm as a device scalar (or float)."""
    if isinstance(optimizer, FusedAdam):
        optimizer.step(max_norm=clip)
        return optimizer.last_norm
    total_norm = calculate_gradient_norm(model)
    torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
    optimizer.step()
    return total_norm


def _post_clip(norm, clip):
    return norm * min(1.0, clip / (norm + 1e-6))


class _Pending:
    """Deferred host read of (loss, norm) of the last queued step."""

    def __init__(self):
        self.item = None

    def push(self, item):
        out, self.item = self.flush(), item
        return out

    def flush(self):
        if self.item is None:
            return None
        vals, meta = self.item
        self.item = None
        host = [v.item() if torch.is_tensor(v) else float(v) for v in vals]
        return host, meta


# ---------------------------------------------------------------------------------------------
def train_one_epoch(epoch, model, dataloader, criterion, optimizer, device, clip, batch_step=0, pbar=None,
                    total_epochs=None, use_amp=False, grad_scaler=None, val_dataloader=None,
                    validation_interval=20):
    """training_utils.py:10-129."""
    if use_amp and grad_scaler is None:
        raise ValueError("use_amp=True but no GradScaler was provided!")
    model.train()
    epoch_loss = 0
    start_time = time.time()
    n_batches = len(dataloader)
    total_steps = total_epochs * n_batches
    gradient_norms = []
    train_steps, train_losses = [], []
    val_steps, val_losses = [], []
    val_iter = iter(val_dataloader) if val_dataloader is not None else None
    pending = _Pending()
    # the next use of the parameters is this loop's forward: the fused optimizer
    # may run its update under that forward (FusedAdam.overlap_next_forward)
    # and nothing in this loop writes the gradients between backward and step, so
    # the clip norm may come from the backward's own epilogue partials
    fused = isinstance(optimizer, FusedAdam) and optimizer._comm is None
    if fused:
        optimizer.overlap_next_forward = True
        optimizer.trust_backward_norm = True

    def report(done):
        nonlocal epoch_loss
        if done is None:
            return
        (loss_v, norm_v), (b_idx, b_step) = done
        train_steps.append(b_step)
        train_losses.append(loss_v)
        print_training_progress(b_idx, norm_v, loss_v, b_step, epoch, total_epochs, n_batches, pbar)
        gradient_norms.append(norm_v)
        epoch_loss += loss_v

    try:
        for batch_idx, (src, trg) in enumerate(dataloader):
            src, trg = src.to(device, non_blocking=True), trg.to(device, non_blocking=True)
            optimizer.zero_grad()
            current_step = batch_step + (epoch * n_batches) + batch_idx
            loss = criterion(model(src), trg, current_step=current_step, total_steps=total_steps)
            loss.backward()
            norm = _step_fused(model, optimizer, clip)
            report(pending.push(((loss.detach(), norm), (batch_idx, batch_step))))
            batch_step += 1
            if val_dataloader is not None and batch_idx % validation_interval == 0:
                report(pending.flush())
                val_iter, vl = _validation_step(model, val_iter, val_dataloader, criterion, device)
                print(f"[Epoch {epoch} - Batch {batch_idx}] Validation Loss: {vl:.4f}")
                val_steps.append(batch_step)
                val_losses.append(vl)
        report(pending.flush())
    finally:
        # reset on every exit, exceptions included: a caller that catches one and
        # then writes p.grad outside autograd must not clip with a stale norm
        if fused:
            optimizer.overlap_next_forward = False
            optimizer.trust_backward_norm = False
            optimizer._sync()
    print_epoch_summary(epoch, total_epochs, epoch_loss, n_batches, time.time() - start_time)
    save_loss_plot(epoch, train_steps, train_losses, val_steps, val_losses, save_dir="dataset/validation_plots/loss")
    save_gradient_norm_plot(epoch, gradient_norms, save_dir="dataset/validation_plots/gradient_norms")
    return batch_step


def _validation_step(model, val_iter, val_dataloader, criterion, device):
    try:
        val_batch = next(val_iter)
    except StopIteration:
        val_iter = iter(val_dataloader)
        val_batch = next(val_iter)
    model.eval()
    with torch.no_grad():
        val_src, val_trg = val_batch
        val_src, val_trg = val_src.to(device), val_trg.to(device)
        val_loss = criterion(model(val_src), val_trg).item()
    model.train()
    return val_iter, val_loss


# ---------------------------------------------------------------------------------------------
def rank_batches(dataloader, rank, world):
    """Yield (step_idx, batch) for the batches rank `rank` of `world` trains on:
    batch s*world + rank of the loader's order, for s < len(loader)//world
    (training_utils.py:160,176-184; leftovers dropped).  Every rank draws the
    same order (same RNG state) but only collates its own batches."""
    steps = len(dataloader) // world
    bs = getattr(dataloader, "batch_sampler", None)
    if bs is None or world == 1:
        it = iter(dataloader)
        for s in range(steps):
            mine = None
            for r in range(world):
                b = next(it)
                if r == rank:
                    mine = b
            yield s, mine
        return
    order = list(bs)
    ds, collate = dataloader.dataset, dataloader.collate_fn
    fetch = getattr(ds, "__getitems__", None)  # batched pinned fetch (dataset.AudioFacialDataset)
    for s in range(steps):
        idx = order[s * world + rank]
        yield s, collate(fetch(idx) if callable(fetch) else [ds[i] for i in idx])


def attach_data_parallel(model, optimizer, world):
    """Wire one rank's engine/optimizer for data parallelism (parallel.py): the
    loss gradient pre-scaled by 1/world, per-rank dropout streams, and one of
    NSTL_DP=zero1_push (default: the sharded optimizer, each shard's slices
    pushed to their owner by the copy engines during backward, no collective
    kernel in it: parallel.ShardPusher), zero1 (the same with a reduce-scatter
    after backward),
    zero1_overlap (each shard reduced onto its owner bucket by bucket during
    backward, the compute stream ceding NSTL_CEDE_CUS CUs, 32 by default (one
    per XCD shader engine), to the collectives) or allreduce (bucketed
    all-reduce during backward, replicated optimizer)."""
    eng = _engine_of(model)
    if eng is None or world == 1 or eng.grad_scale_t is not None:
        return
    eng.grad_scale_t = torch.full((1,), 1.0 / world, device=eng.device)
    eng.seed_salt = dist.get_rank()
    mode = os.environ.get("NSTL_DP", "zero1_push")
    if mode == "allreduce" or not hasattr(optimizer, "shard"):
        from ..parallel import GradAllReducer
        eng.grad_reducer = GradAllReducer(eng.g32)
    else:
        optimizer.shard()
        if mode == "zero1_push":
            from ..parallel import ShardPusher
            # None: zero1 (every rank agrees); gather: the bf16 weight arena the
            # sharded step all-gathers (parallel.zero1_step)
            eng.grad_reducer = ShardPusher.create(eng.g32, optimizer._comm,
                                                  gather=[eng.p16 if eng.p16 is not eng.p32 else eng.p32])
            if eng.grad_reducer is None:
                optimizer.dp_fallback = "zero1_push -> zero1 (setup: IPC mapping or copy-engine self-test failed)"
        elif mode == "zero1_overlap":
            from ..parallel import GradShardReducer, cede_cus
            cede_cus(int(os.environ.get("NSTL_CEDE_CUS", "32")), eng.device)
            eng.grad_reducer = GradShardReducer(eng.g32, optimizer._comm)


def gradient_exchange(model, optimizer):
    """The gradient exchange a rank is running now (after attach_data_parallel;
    it can change after the first step, see ShardPusher.verify): "zero1_push",
    "zero1_overlap", "allreduce", "zero1" (the post-backward reduce-scatter), or
    None (one process)."""
    eng = _engine_of(model)
    if eng is None or eng.grad_scale_t is None:
        return None
    red = eng.grad_reducer
    if red is not None and red.active:
        return red.mode
    return "zero1" if getattr(optimizer, "_comm", None) is not None else "allreduce"


def train_one_epoch_multi_gpu(epoch, models, dataloader, criterion, optimizer, devices, clip, batch_step=0,
                              pbar=None, total_epochs=None, use_amp=False, grad_scaler=None, val_dataloader=None,
                              validation_interval=20):
    """training_utils.py:131-303.  Under torch.distributed each rank passes
    [its model] / [its device]; without it, a list of in-process replicas."""
    if use_amp and grad_scaler is None:
        raise ValueError("use_amp=True but no GradScaler was provided!")
    models = list(models) if isinstance(models, (list, tuple)) else [models]
    devices = list(devices) if isinstance(devices, (list, tuple)) else [devices]
    rank, world = _dist()
    if world > 1 and len(models) != 1:
        raise ValueError("under torch.distributed pass this rank's model only (got %d)" % len(models))
    n = world if world > 1 else len(models)
    steps_per_epoch = len(dataloader) // n
    total_steps = total_epochs * steps_per_epoch
    epoch_loss = 0
    gradient_norms = []
    train_steps, train_losses = [], []
    val_steps, val_losses = [], []
    val_iter = iter(val_dataloader) if val_dataloader is not None else None
    start_time = time.time()
    for m in models:
        m.train()
    if world > 1:
        attach_data_parallel(models[0], optimizer, world)
    pending = _Pending()

    def report(done):
        nonlocal epoch_loss
        if done is None:
            return
        (loss_v, norm_v), (s_idx, b_step) = done
        if rank == 0:
            print_training_progress(s_idx, norm_v, loss_v, b_step, epoch, total_epochs, steps_per_epoch, pbar)
        gradient_norms.append(norm_v)
        epoch_loss += loss_v
        train_steps.append(b_step)
        train_losses.append(loss_v)
        gradient_norms.append(_post_clip(norm_v, clip))

    if world > 1:
        batches = rank_batches(dataloader, rank, world)
    else:
        batches = _grouped(dataloader, n)
    for step_idx, batch in batches:
        current_step = batch_step + (epoch * steps_per_epoch) + step_idx
        optimizer.zero_grad()
        if world > 1:
            src, trg = batch
            src, trg = src.to(devices[0], non_blocking=True), trg.to(devices[0], non_blocking=True)
            loss = criterion(models[0](src), trg, current_step=current_step, total_steps=total_steps)
            loss.backward()  # bucketed RCCL all-reduce runs inside (engine.backward)
            if _engine_of(models[0]) is None:
                _allreduce_mean_grads(models[0], world)
            norm = _step_fused(models[0], optimizer, clip)
            mean_loss = loss.detach().clone()
            dist.all_reduce(mean_loss)
            mean_loss /= world
        else:
            losses = []
            for i in range(n):
                src, trg = batch[i]
                src, trg = src.to(devices[i], non_blocking=True), trg.to(devices[i], non_blocking=True)
                if i > 0:
                    models[i].zero_grad(set_to_none=False) if _engine_of(models[i]) is None else \
                        _engine_of(models[i]).zero_grad()
                loss_i = criterion(models[i](src), trg, current_step=current_step, total_steps=total_steps)
                loss_i.backward()
                losses.append(loss_i.detach())
            _average_into_primary(models, devices)
            norm = _step_fused(models[0], optimizer, clip)
            _broadcast_from_primary(models)
            mean_loss = sum(l.to(devices[0]) for l in losses) / n
        report(pending.push(((mean_loss, norm), (step_idx, batch_step))))
        batch_step += 1
        if val_dataloader is not None and step_idx % validation_interval == 0:
            report(pending.flush())
            if rank == 0:
                val_iter, vl = _validation_step(models[0], val_iter, val_dataloader, criterion, devices[0])
                print(f"[Epoch {epoch} - Step {step_idx}] Validation Loss: {vl:.4f}")
                val_steps.append(batch_step)
                val_losses.append(vl)
        if pbar is not None:
            pbar.update(1)
    report(pending.flush())
    if rank == 0:
        print_epoch_summary(epoch, total_epochs, epoch_loss, steps_per_epoch, time.time() - start_time)
        save_gradient_norm_plot(epoch, gradient_norms, save_dir="dataset/validation_plots/gradient_norms")
        save_loss_plot(epoch, train_steps, train_losses, val_steps, val_losses, save_dir="dataset/validation_plots/loss")
    return batch_step


def _allreduce_mean_grads(model, world):
    """Gradient mean for a module without the engine's in-backward reducer."""
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat)
    flat /= world
    o = 0
    for g in grads:
        g.copy_(flat[o:o + g.numel()].view_as(g))
        o += g.numel()


def _grouped(dataloader, n):
    it = iter(dataloader)
    for s in range(len(dataloader) // n):
        group = []
        try:
            for _ in range(n):
                group.append(next(it))
        except StopIteration:
            print(f"Dropping leftover mini-batches at step {s}.")
            return
        yield s, group


def _average_into_primary(models, devices):
    """training_utils.py:228-235 on flat arenas: grad0 = mean_i grad_i."""
    e0 = _engine_of(models[0])
    with torch.no_grad():
        if e0 is not None and all(_engine_of(m) is not None for m in models):
            e0.invalidate_sq()
            for m in models[1:]:
                e0.g32.add_(_engine_of(m).g32.to(e0.device, non_blocking=True))
            e0.g32.div_(len(models))
            return
        for group in zip(*[m.parameters() for m in models]):
            if all(p.grad is not None for p in group):
                avg = sum(p.grad.to(devices[0]) for p in group) / len(models)
                group[0].grad.copy_(avg.view_as(group[0]))


def _broadcast_from_primary(models):
    """training_utils.py:254-263: replicas take models[0]'s parameters."""
    e0 = _engine_of(models[0])
    with torch.no_grad():
        for m in models[1:]:
            e = _engine_of(m)
            if e0 is not None and e is not None:
                e.p32.copy_(e0.p32.to(e.device, non_blocking=True))
                e.refresh_shadow()
            else:
                for p0, p in zip(models[0].parameters(), m.parameters()):
                    p.copy_(p0.to(p.device))


# ---------------------------------------------------------------------------------------------
def save_loss_plot(epoch, train_steps, train_losses, val_steps, val_losses, save_dir="dataset/validation_plots/loss"):
    """training_utils.py:309-332."""
    plt = _pyplot()
    os.makedirs(save_dir, exist_ok=True)
    plt.figure(figsize=(10, 6))
    plt.plot(train_steps, train_losses, label="Training Loss", marker='o', markersize=3)
    plt.plot(val_steps, val_losses, label="Validation Loss", marker='x', markersize=8, linestyle='--')
    plt.xlabel("Training Step")
    plt.ylabel("Loss")
    plt.title(f"Loss Values (Epoch {epoch + 1})")
    plt.legend()
    plt.grid(True)
    plot_path = os.path.join(save_dir, f"loss_epoch_{epoch + 1}.png")
    plt.savefig(plot_path)
    plt.close()
    print(f"Loss plot saved to {plot_path}")


def init_weights(m):
    """training_utils.py:336-341: N(0, 0.02) weights, zero biases (Linear/Conv1d)."""
    if isinstance(m, (nn.Linear, nn.Conv1d)):
        print(f"Initializing {m} with normal distribution")
        nn.init.normal_(m.weight, mean=0.0, std=0.02)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)


def count_parameters(model):
    param_count = sum(p.numel() for p in model.parameters())
    print(f"Total number of parameters: {param_count}")
    return param_count


def calculate_gradient_norm(model):
    """training_utils.py:349-357 (global L2 norm of the gradients, a float).
    With the engine: one reduction over the flat gradient arena."""
    eng = _engine_of(model)
    if eng is not None:
        return math.sqrt(float(eng.g32[:eng.numel].double().pow(2).sum().item()))
    total = 0.0
    for p in model.parameters():
        if p.grad is not None:
            total += p.grad.detach().norm(2).item() ** 2
    return total ** 0.5


def print_training_progress(batch_idx, total_norm, batch_loss, batch_step, epoch, total_epochs, dataloader_len, pbar):
    """training_utils.py:359-364."""
    print(f"Batch {batch_idx}, Gradient Norm: {total_norm}")
    if pbar is not None:
        pbar.update(1)
    total = pbar.total if pbar is not None else None
    print(f"Step [{batch_step}/{total}], Epoch [{epoch + 1}/{total_epochs}], Batch [{batch_idx + 1}/{dataloader_len}], "
          f"Current Loss: {batch_loss:.4f}")


def print_epoch_summary(epoch, total_epochs, epoch_loss, dataloader_len, epoch_time):
    print(f"Epoch [{epoch + 1}/{total_epochs}], Loss: {epoch_loss / max(1, dataloader_len):.4f}, "
          f"Time: {epoch_time:.2f} seconds")


def save_gradient_norm_plot(epoch, gradient_norms, save_dir):
    """training_utils.py:370-383."""
    plt = _pyplot()
    os.makedirs(save_dir, exist_ok=True)
    plt.figure(figsize=(10, 6))
    plt.plot(gradient_norms, label="Gradient Norm")
    plt.xlabel("Batch Index")
    plt.ylabel("Gradient Norm")
    plt.title(f"Gradient Norm Fluctuations (Epoch {epoch + 1})")
    plt.legend()
    plt.grid(True)
    plot_path = os.path.join(save_dir, f"gradient_norms_epoch_{epoch + 1}.png")
    plt.savefig(plot_path)
    plt.close()
    print(f"Gradient norm plot saved to {plot_path}")


def _pyplot():
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    return plt
