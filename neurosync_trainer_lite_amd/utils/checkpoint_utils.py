"""Drop-in for utils/checkpoint_utils.py:10-57: same checkpoint dict
({'model_state_dict', 'optimizer_state_dict', 'scheduler_state_dict', 'epoch',
'batch_step', 'config'}), same backup rotation (the previous checkpoint moves to
backup_<timestamp>/, the 5 newest backups are kept), same return tuple.  Loading
uses ``weights_only=True`` (no code runs from the file); reference checkpoints
load unchanged."""
import os
import shutil
from datetime import datetime

import torch


def save_checkpoint(model, optimizer, scheduler, epoch, batch_step, config):
    checkpoint = {
        'model_state_dict': model.state_dict(),
        'optimizer_state_dict': optimizer.state_dict(),
        'scheduler_state_dict': scheduler.state_dict(),
        'epoch': epoch,
        'batch_step': batch_step,
        'config': config,
    }
    checkpoint_path = config['checkpoint_path']
    ckpt_dir = os.path.dirname(checkpoint_path)
    if ckpt_dir:
        os.makedirs(ckpt_dir, exist_ok=True)
    if os.path.exists(checkpoint_path):
        stamp = datetime.now().strftime('%Y%m%d_%H%M%S')
        backup_dir = os.path.join(ckpt_dir, f"backup_{stamp}")
        suffix = 1
        while os.path.exists(backup_dir):  # two saves within one second
            backup_dir = os.path.join(ckpt_dir, f"backup_{stamp}_{suffix}")
            suffix += 1
        os.makedirs(backup_dir)
        shutil.move(checkpoint_path, os.path.join(backup_dir, os.path.basename(checkpoint_path)))
        base = ckpt_dir or "."
        backups = sorted((d for d in os.listdir(base) if d.startswith("backup_")),
                         key=lambda d: os.path.getmtime(os.path.join(base, d)), reverse=True)
        for old in backups[5:]:
            shutil.rmtree(os.path.join(base, old))
    torch.save(checkpoint, checkpoint_path)


def load_checkpoint(checkpoint_path, model, optimizer, scheduler, device):
    checkpoint = torch.load(checkpoint_path, map_location=device, weights_only=True)
    model.load_state_dict(checkpoint['model_state_dict'])
    optimizer.load_state_dict(checkpoint['optimizer_state_dict'])
    scheduler.load_state_dict(checkpoint['scheduler_state_dict'])
    return checkpoint['epoch'], checkpoint['batch_step'], model, optimizer, scheduler


def save_checkpoint_and_data(epoch, model, optimizer, scheduler, batch_step, config, lock, device):
    """checkpoint_utils.py:53-57: checkpoint, model.pth, then the per-epoch
    validation clip (utils/validation.py)."""
    from .validation import generate_and_save_facial_data
    save_checkpoint(model, optimizer, scheduler, epoch, batch_step, config)
    model_dir = os.path.dirname(config['model_path'])
    if model_dir:
        os.makedirs(model_dir, exist_ok=True)
    torch.save(model.state_dict(), config['model_path'])
    generate_and_save_facial_data(epoch, config['audio_path'], model, config['ground_truth_path'], lock, device)
