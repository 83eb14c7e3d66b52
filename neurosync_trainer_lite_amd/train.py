"""Drop-in for train.py (train_model + entry point), MI355X data-parallel.

    python -m neurosync_trainer_lite_amd.train                 # 1 GPU
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 -m neurosync_trainer_lite_amd.train

With ``use_multi_gpu`` and ``num_gpus`` > 1 but no torchrun environment, the
entry point starts torch.distributed.run as a child process (one process per
GPU, RCCL over xGMI) instead of the reference's single-process replicas
(train.py:62-78, at most 4 GPUs).  Every rank builds the same datasets and the
same batch order from one broadcast seed, trains on batches r, r+n, ...;
rank 0 alone writes checkpoints, plots and the validation clip.
"""
import json
import os
import socket
import subprocess
import sys
import tempfile
import threading

import torch
import torch.distributed as dist

from . import parallel
from .config import training_config
from .dataset.dataset import prepare_dataloader_with_split
from .utils.checkpoint_utils import load_checkpoint, save_checkpoint_and_data
from .utils.model_utils import build_model, prepare_training_components, save_final_model
from .utils.training_utils import count_parameters, init_weights, train_one_epoch, train_one_epoch_multi_gpu


class _NoScaler:
    """Stands in for torch.cuda.amp.GradScaler (train.py:26): bf16 needs no loss
    scaling; train_one_epoch only checks that one was given."""

    def state_dict(self):
        return {}


def train_model(config, model_0, model_1, model_2, model_3, dataloader, val_dataloader, criterion, optimizer,
                scheduler, devices, use_multi_gpu=False, start_epoch=0, batch_step=0):
    """train.py:12-58."""
    n_epochs = config['n_epochs']
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist.is_initialized() else (0, 1)
    lock = threading.Lock()
    if rank == 0:
        count_parameters(model_0)
    device0 = devices[0]
    use_amp = config.get('use_amp', True)
    scaler = _NoScaler() if use_amp else None
    pbar = None
    if rank == 0:
        from tqdm import tqdm
        steps = len(dataloader) // max(1, world) if world > 1 else len(dataloader)
        pbar = tqdm(total=n_epochs * steps, desc="Training", dynamic_ncols=True)
    try:
        for epoch in range(start_epoch, n_epochs):
            if use_multi_gpu:
                models, used = [model_0], [devices[0]]
                if world == 1:
                    for m, d in ((model_1, devices[1]), (model_2, devices[2]), (model_3, devices[3])):
                        if m is not None:
                            models.append(m)
                            used.append(d)
                batch_step = train_one_epoch_multi_gpu(epoch, models, dataloader, criterion, optimizer, used,
                                                       clip=2.0, batch_step=batch_step, pbar=pbar,
                                                       total_epochs=n_epochs, use_amp=use_amp, grad_scaler=scaler,
                                                       val_dataloader=val_dataloader, validation_interval=20)
            else:
                batch_step = train_one_epoch(epoch, model=model_0, dataloader=dataloader, criterion=criterion,
                                             optimizer=optimizer, device=device0, clip=2.0, batch_step=batch_step,
                                             pbar=pbar, total_epochs=n_epochs, use_amp=use_amp, grad_scaler=scaler,
                                             val_dataloader=val_dataloader, validation_interval=20)
            scheduler.step()
            if world > 1 and hasattr(optimizer, "consolidate"):
                optimizer.consolidate()  # sharded optimizer: every rank, before rank 0 saves
            if rank == 0:
                save_checkpoint_and_data(epoch, model_0, optimizer, scheduler, batch_step, config, lock, device0)
            if world > 1:
                dist.barrier()
        if world > 1 and hasattr(optimizer, "consolidate"):
            optimizer.consolidate()
        if rank == 0:
            save_final_model(model_0)
    finally:
        if pbar is not None:
            pbar.close()
    return batch_step


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


CONFIG_ENV = "NSTL_TRAIN_CONFIG"


def _relaunch(n, config):
    """torchrun this module on n GPUs with ``config`` handed over as a JSON file
    (its path in $NSTL_TRAIN_CONFIG), so the children train the caller's config
    rather than the module default."""
    with tempfile.NamedTemporaryFile("w", suffix=".json", prefix="nstl_config_", delete=False) as f:
        json.dump(config, f)
        path = f.name
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m", "neurosync_trainer_lite_amd.train"]
    try:
        return subprocess.call(cmd, env=dict(os.environ, **{CONFIG_ENV: path}))
    finally:
        os.unlink(path)


def _config_from_env():
    path = os.environ.get(CONFIG_ENV)
    if not path:
        return None
    with open(path) as f:
        return json.load(f)


def _common_seed(rank, world, device):
    seed = torch.tensor([int.from_bytes(os.urandom(7), "little") if rank == 0 else 0], dtype=torch.int64,
                        device=device)
    if world > 1:
        dist.broadcast(seed, 0)
    return int(seed.item())


def main(config=None):
    config = dict(training_config if config is None else config)
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    n_dev = torch.cuda.device_count()
    if world_env == 1 and config.get('use_multi_gpu', False) and n_dev > 1 and config.get('num_gpus', 1) > 1:
        return _relaunch(min(n_dev, config['num_gpus']), config)
    if n_dev == 0:
        raise RuntimeError("the MI355X training path needs a GPU (there is no CPU path)")
    rank, world, local = parallel.init_from_env()
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)
    seed = _common_seed(rank, world, device)
    torch.manual_seed(seed)  # same datasets split and initial weights on every rank
    train_dataset, val_dataset, train_dataloader, val_dataloader = prepare_dataloader_with_split(config, val_split=0.1)
    if world > 1 and hasattr(train_dataloader.sampler, "generator"):
        train_dataloader.sampler.generator = torch.Generator().manual_seed(seed)
    use_multi_gpu = world > 1
    devices = [device, None, None, None]
    model_0 = build_model(config, device)
    criterion, optimizer, scheduler = prepare_training_components(config, model_0)
    start_epoch, batch_step = 0, 0
    if config['mode'] == 'resume' and os.path.exists(config['checkpoint_path']):
        start_epoch, batch_step, model_0, optimizer, scheduler = load_checkpoint(
            config['checkpoint_path'], model_0, optimizer, scheduler, device)
    else:
        model_0.apply(init_weights)
    if world > 1:
        eng = model_0.engine()
        dist.broadcast(eng.p32, 0)
        eng.refresh_shadow()
    return train_model(config, model_0, None, None, None, train_dataloader, val_dataloader, criterion, optimizer,
                       scheduler, devices, use_multi_gpu=use_multi_gpu, start_epoch=start_epoch, batch_step=batch_step)


if __name__ == "__main__":
    main(_config_from_env())
